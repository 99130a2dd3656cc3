"""Data-parallel path on CPU with gloo, world_size 2 (the real RCCL path runs on the GPU box).

DP equivalence: with equal per-rank batches, averaging per-rank gradients of the
per-rank mean loss equals the gradient of the loss over the concatenated batch, because every
normalisation in video_net is per sample.  The reducer under test is the product's
GradAllReducer operating on a flat gradient buffer; the model is the CPU oracle.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat_grads(model):
    return torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.requires_grad])


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from cesm_emulator_amd import distributed as D
    from oracle import ref_cpu as R
    D.setup(backend="gloo")
    torch.manual_seed(1)
    net = R.UNet(base_ch=64, ch_mults=(1, 2))
    d = R.Diffusion(net)
    red = D.GradAllReducer(bucket_bytes=1 << 20)
    # replicas start identical after the broadcast even if a rank perturbs its copy
    flat = torch.nn.utils.parameters_to_vector([p for p in net.parameters() if p.requires_grad])
    if rank == 1:
        flat = flat + 1.0
    red.broadcast_params(flat)
    torch.nn.utils.vector_to_parameters(flat, [p for p in net.parameters() if p.requires_grad])
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(4, 1, 16, 24, generator=g)
    cond = torch.randn(4, 1, 3, 16, 24, generator=g)
    t = torch.randint(0, 1000, (4,), generator=g)
    noise = torch.randn(4, 1, 16, 24, generator=g)
    sl = slice(2 * rank, 2 * rank + 2)
    d.loss(x0[sl], cond[sl], t=t[sl], noise=noise[sl]).backward()
    fg = _flat_grads(net)
    red.allreduce_grads(fg)
    if rank == 0:
        torch.save({"dp": fg, "params": flat}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_equals_full_batch(tmp_path):
    out = str(tmp_path / "dp.pt")
    port = _free_port()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    from oracle import ref_cpu as R
    torch.manual_seed(1)
    net = R.UNet(base_ch=64, ch_mults=(1, 2))
    torch.testing.assert_close(torch.nn.utils.parameters_to_vector(
        [p for p in net.parameters() if p.requires_grad]), res["params"])
    d = R.Diffusion(net)
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(4, 1, 16, 24, generator=g)
    cond = torch.randn(4, 1, 3, 16, 24, generator=g)
    t = torch.randint(0, 1000, (4,), generator=g)
    noise = torch.randn(4, 1, 16, 24, generator=g)
    d.loss(x0, cond, t=t, noise=noise).backward()
    full = _flat_grads(net)
    rel = ((res["dp"] - full).norm() / full.norm()).item()
    assert rel < 1e-5, rel


def test_bucketing_covers_buffer():
    from cesm_emulator_amd.distributed import GradAllReducer
    r = GradAllReducer(bucket_bytes=4 * 10)
    b = r.buckets(95)
    assert b[0] == (0, 10) and b[-1] == (90, 95)
    assert sum(e - s for s, e in b) == 95


def _overlap_worker(rank, world, port, out_path):
    """The overlapped path: buckets are reduced from the end of the flat buffer as the backward
    reports parameter groups final (reverse construction order), the rest in finish()."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from types import SimpleNamespace
    from cesm_emulator_amd import distributed as D
    D.setup(backend="gloo")
    sizes = [7, 130, 64, 300, 5, 90]
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + 63) // 64 * 64
    g = torch.zeros(o)
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    gen = torch.Generator().manual_seed(100 + rank)
    for n, off in zip(sizes, offs):
        g[off:off + n] = torch.randn(n, generator=gen)
    flat = SimpleNamespace(params=params, offsets=offs, grad=g)
    net = SimpleNamespace(_grad_ready=None)
    red = D.GradAllReducer(bucket_bytes=4 * 100)
    red.arm(net, flat)
    issued = []
    for grp in ([5], [4, 3], [2], [1]):  # reverse construction order; param 0 is the shared one
        net._grad_ready([params[i] for i in grp])
        issued.append(red._armed["lo"])
    red.finish(net)
    torch.save({"g": g, "issued": torch.tensor(issued)}, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_allreduce_matches_average(tmp_path):
    out = str(tmp_path / "ov.pt")
    mp.spawn(_overlap_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    torch.testing.assert_close(r0["g"], r1["g"])
    sizes = [7, 130, 64, 300, 5, 90]
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + 63) // 64 * 64
    exp = torch.zeros(o)
    for rank in (0, 1):
        gen = torch.Generator().manual_seed(100 + rank)
        for n, off in zip(sizes, offs):
            exp[off:off + n] += torch.randn(n, generator=gen) / 2
    torch.testing.assert_close(r0["g"], exp)
    lo = r0["issued"].tolist()
    # buckets went out before finish(): after the last group only the shared param's bucket is left
    assert lo[0] < o and lo[-1] <= 64 and lo == sorted(lo, reverse=True), lo


def _seed_worker(rank, world, port, out_path):
    """train_one_epoch's data-parallel branch on CPU (gloo): each rank gets its own t / eps stream from a base
    seed broadcast by rank 0 (the ranks' default generators deliberately differ here) and dp.rank"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from types import SimpleNamespace
    from cesm_emulator_amd import distributed as D
    from cesm_emulator_amd.train import train_one_epoch
    D.setup(backend="gloo")
    torch.manual_seed(50 + rank)  # diverged default generators: the broadcast base seed must still agree
    red = D.GradAllReducer()
    diff = SimpleNamespace(train=lambda: None, model=SimpleNamespace(), generator=None)
    train_one_epoch(diff, [], None, torch.device("cpu"), dp=red)  # empty loader: only the set-up runs
    t = torch.randint(0, 1000, (16,), generator=diff.generator)
    eps = torch.randn(16, generator=diff.generator)
    torch.save({"t": t, "eps": eps, "seed": diff.generator.initial_seed(), "rank": red.rank}, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_train_one_epoch_rank_streams(tmp_path):
    out = str(tmp_path / "seed.pt")
    mp.spawn(_seed_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    assert (r0["rank"], r1["rank"]) == (0, 1)
    assert r1["seed"] == r0["seed"] + 1  # one broadcast base seed, offset by the all-reducer's rank
    assert not torch.equal(r0["t"], r1["t"]) and not torch.equal(r0["eps"], r1["eps"])
