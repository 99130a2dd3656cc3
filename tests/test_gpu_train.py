"""Training-loop plumbing on the GPU: the data path feeding real steps (A17 / F2), the optimizer's
device step counter, per-forward backward tapes, per-rank t / eps streams and the data-parallel step
through the product's train_step + GradAllReducer (2 ranks, gloo, one GPU).

Reference: dataset_single_member.py:168-196 (item), train.py:1005-1012 / 830-831 (DataLoader, pin,
H2D), train.py:849-880 (step), model.py:205-206 (t / eps draws), SURVEY.md §8(e) E1.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from cesm_emulator_amd import data as DA
from cesm_emulator_amd.model import UNet, Diffusion
from cesm_emulator_amd.optim import FusedAdamW
from cesm_emulator_amd.train import train_step, train_one_epoch, rank_generator

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b).clamp_min(1e-30)).item()


def _fields(T=10, M=3, H=20, W=24, seed=0):
    r = np.random.default_rng(seed)
    return r.standard_normal((T, M, H, W)).astype(np.float32), r.standard_normal((T, M, H, W)).astype(np.float32)


# ------------------------------------------------------------------ data path vs the dataset restatement
@pytest.mark.parametrize("kind", ["pinned", "device"])
@pytest.mark.parametrize("center", [True, False])
@pytest.mark.parametrize("crop", [None, (16, 16)])
@pytest.mark.parametrize("p", [0.0, 0.5, 1.0])
def test_loader_batches_bit_equal_to_dataset(dev, kind, center, crop, p):
    """every batch the loader yields == the reference dataset's items for the same indices under the same
    numpy seed (time reversal, crop draws in __getitem__ order), bit for bit"""
    from oracle.ref_data import WindowedAllMembersDatasetRef
    cond, tgt = _fields()
    Kw, bs = 5, 4
    ref = WindowedAllMembersDatasetRef(cond[:, :, None], tgt[:, :, None], K=Kw, center=center, crop_hw=crop,
                                       time_reverse_p=p)
    cls = DA.PinnedWindowLoader if kind == "pinned" else DA.DeviceWindowLoader
    ld = cls(cond, tgt, Kw, bs, dev, center=center, crop_hw=crop, time_reverse_p=p, shuffle=True, seed=3)
    ld.set_epoch(1)
    batches = DA.shard_indices(len(ref), bs, 0, 1, True, 3, 1)
    np.random.seed(123)
    got = [(c.clone(), x.clone()) for c, x in ld]
    np.random.seed(123)
    assert len(got) == len(batches)
    for (c, x), idx in zip(got, batches):
        items = [ref[i] for i in idx]
        c_ref = torch.stack([a for a, _ in items])
        x_ref = torch.stack([b for _, b in items])
        assert torch.equal(c.cpu(), c_ref) and torch.equal(x.cpu(), x_ref)


def test_loaders_feed_training_identically(dev):
    """train_one_epoch fed by the pinned (host gather + side-stream H2D) and the device (HBM gather) loader
    gives identical epoch losses and parameters (same numpy / t-eps seeds), bit-identical in fp32 and in bf16
    mode (every reduction on the bf16 path has a fixed order, tests/test_gpu_determinism.py)"""
    cond, tgt = _fields(T=8, M=2, H=32, W=48, seed=1)
    Kw = 3
    out = {}
    for dt in ("fp32", "bf16"):
        for kind in ("pinned", "device"):
            torch.manual_seed(0)
            net = UNet(ch_mults=(1, 2)).to(dev)
            d = Diffusion(net).to(dev)
            d.generator = rank_generator(dev, 2, 0)
            opt = FusedAdamW(d.parameters(), lr=1e-3, max_grad_norm=1.0)
            cls = DA.PinnedWindowLoader if kind == "pinned" else DA.DeviceWindowLoader
            ld = cls(cond, tgt, Kw, 4, dev, crop_hw=(32, 32), time_reverse_p=0.5, seed=0)
            np.random.seed(7)
            loss = train_one_epoch(d, ld, opt, dev, 1.0, use_amp=(dt == "bf16"))
            torch.cuda.synchronize()
            out[(dt, kind)] = (loss, opt.flat.data.clone())
        lp, pp = out[(dt, "pinned")]
        ldv, pd = out[(dt, "device")]
        print(f"{dt}: epoch loss pinned {lp:.6f} device {ldv:.6f}, params rel {rel(pp, pd):.2e}")
        assert np.isfinite(lp)
        assert lp == ldv and torch.equal(pp, pd)


# ------------------------------------------------------------------ optimizer / autograd / RNG plumbing
def test_nonfinite_step_is_skipped_and_not_counted(dev):
    """a non-finite loss skips the update on device and does NOT advance the step counter, so the next
    finite step uses step-1 bias corrections, as torch.optim.AdamW would (it never sees the bad step)"""
    torch.manual_seed(8)
    ps = [torch.randn(37, 5), torch.randn(1000)]
    g = [torch.randn_like(p) for p in ps]
    ref = [p.clone().double().requires_grad_(True) for p in ps]
    opt_r = torch.optim.AdamW(ref, lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)
    dp = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
    opt = FusedAdamW(dp, lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=None)
    before = opt.flat.data.clone()
    for p, gg in zip(dp, g):
        p.grad.copy_(gg.to(dev))
    opt.step(loss=torch.tensor([float("nan")], device=dev))
    assert opt.step_count == 0 and torch.equal(opt.flat.data, before)
    assert opt.state_dict()["state"] == {}
    for p, gg in zip(dp, g):
        p.grad.copy_(gg.to(dev))
    opt.step(loss=torch.tensor([1.0], device=dev))
    for r, gg in zip(ref, g):
        r.grad = gg.double().clone()
    opt_r.step()
    assert opt.step_count == 1
    for p, r in zip(dp, ref):
        assert rel(p.detach(), r.detach()) < 1e-6
    assert float(opt.state_dict()["state"][0]["step"]) == 1.0


def test_nan_in_cond_skips_bf16_train_step(dev):
    """the reference's guard (train.py:860-861) on the production path: a NaN at ONE pixel of one frame of `cond`
    in a bf16 train_step (more_blocks mults, F = 12, 64 x 96: the fused level-0 attention kernels, built without
    NaN semantics, build.py NO_NANS) must surface as a non-finite loss, skip the AdamW step on device and leave
    every parameter and the optimizer state untouched; the next clean step then trains normally"""
    torch.manual_seed(3)
    net = UNet(ch_mults=(1, 2, 4, 8)).to(dev)
    net.compute_dtype = torch.bfloat16
    d = Diffusion(net).to(dev)
    opt = FusedAdamW(d.parameters(), lr=1e-3, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(9)
    x0 = torch.randn(1, 1, 64, 96, generator=g).to(dev)
    cond = torch.randn(1, 1, 12, 64, 96, generator=g).to(dev)
    t = torch.randint(0, 1000, (1,), generator=g).to(dev)
    noise = torch.randn(1, 1, 64, 96, generator=g).to(dev)
    bad = cond.clone()
    bad[0, 0, 7, 40, 13] = float("nan")
    before = opt.flat.data.clone()
    loss = train_step(d, opt, x0, bad, 1.0, t=t, noise=noise)
    torch.cuda.synchronize()
    assert not torch.isfinite(loss).all(), float(loss)
    assert opt.step_count == 0 and torch.equal(opt.flat.data, before)
    assert opt.state_dict()["state"] == {}
    loss = train_step(d, opt, x0, cond, 1.0, t=t, noise=noise)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all() and opt.step_count == 1
    assert torch.isfinite(opt.flat.data).all() and not torch.equal(opt.flat.data, before)


def test_two_forwards_then_one_backward(dev):
    """each forward's autograd node owns its backward tape: (loss(a) + loss(b)).backward() == the sum of
    the separate gradients, and l1.backward() after a second forward replays l1's activations"""
    torch.manual_seed(0)
    net = UNet(ch_mults=(1, 2)).to(dev)
    net.compute_dtype = torch.float32
    d = Diffusion(net).to(dev)
    g = torch.Generator().manual_seed(4)
    mk = lambda: [torch.randn(2, 1, 16, 24, generator=g).to(dev), torch.randn(2, 1, 3, 16, 24, generator=g).to(dev),
                  torch.randint(0, 1000, (2,), generator=g).to(dev), torch.randn(2, 1, 16, 24, generator=g).to(dev)]
    a, b = mk(), mk()

    def grads(fn):
        for p in d.parameters():
            p.grad = None
        fn()
        return {n: p.grad.clone() for n, p in d.named_parameters() if p.grad is not None}

    ga = grads(lambda: d.loss(a[0], a[1], t=a[2], noise=a[3]).backward())
    gb = grads(lambda: d.loss(b[0], b[1], t=b[2], noise=b[3]).backward())
    gs = grads(lambda: (d.loss(a[0], a[1], t=a[2], noise=a[3]) + d.loss(b[0], b[1], t=b[2], noise=b[3])).backward())

    def first_after_second():
        l1 = d.loss(a[0], a[1], t=a[2], noise=a[3])
        d.loss(b[0], b[1], t=b[2], noise=b[3])  # a second grad-enabled forward, never backpropagated
        l1.backward()

    g1 = grads(first_after_second)
    for n in ga:
        assert rel(gs[n], ga[n] + gb[n]) < 1e-5, n
        assert rel(g1[n], ga[n]) < 1e-6, n


def test_rank_generators_give_distinct_draws(dev):
    """per-rank t / eps streams (seed + rank): reproducible per rank, different across ranks"""
    d = Diffusion(torch.nn.Identity()).to(dev)
    x0 = torch.zeros(8, 1, 4, 4, device=dev)

    def draw(rank):
        d.generator = rank_generator(dev, 2, rank)
        B = x0.shape[0]
        t = torch.randint(0, d.T, (B,), device=dev, generator=d.generator)
        n = torch.randn(x0.shape, device=dev, generator=d.generator)
        return t, n

    t0, n0 = draw(0)
    t0b, n0b = draw(0)
    t1, n1 = draw(1)
    assert torch.equal(t0, t0b) and torch.equal(n0, n0b)
    assert not torch.equal(t0, t1) and not torch.equal(n0, n1)


# ------------------------------------------------------------------ data parallel through the product step
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    g = torch.Generator().manual_seed(11)
    x0 = torch.randn(4, 1, 16, 24, generator=g)
    cond = torch.randn(4, 1, 3, 16, 24, generator=g)
    t = torch.randint(0, 1000, (4,), generator=g)
    noise = torch.randn(4, 1, 16, 24, generator=g)
    return x0, cond, t, noise


def _make(dev, dtype=torch.float32):
    torch.manual_seed(1)
    net = UNet(ch_mults=(1, 2)).to(dev)
    net.compute_dtype = dtype
    d = Diffusion(net).to(dev)
    opt = FusedAdamW(d.parameters(), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    return d, opt


def _dp_worker(rank, world, port, out_path, dtype=torch.float32):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from cesm_emulator_amd import distributed as D
    torch.cuda.set_device(0)
    D.setup(backend="gloo")
    dev = torch.device("cuda:0")
    d, opt = _make(dev, dtype)
    red = D.GradAllReducer(bucket_bytes=256 << 10)
    if rank == 1:  # a perturbed replica is re-synchronised by the initial broadcast
        opt.flat.data.add_(1.0)
    red.broadcast_params(opt.flat.data)
    x0, cond, t, noise = _batch()
    sl = slice(2 * rank, 2 * rank + 2)
    for _ in range(2):
        train_step(d, opt, x0[sl].to(dev), cond[sl].to(dev), 1.0, red, t=t[sl].to(dev), noise=noise[sl].to(dev))
    torch.cuda.synchronize()
    torch.save(opt.flat.data.cpu(), f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_dp_step_equals_full_batch_step(dev, tmp_path, dtype):
    """2 ranks (gloo on one GPU) through train_step + GradAllReducer.arm/finish (overlapped buckets) with
    explicit t / eps: after two steps both replicas equal the 1-rank run on the concatenated batch, in the fp32
    kernel mode and on the bf16 production kernels"""
    port = _free_port()
    out = str(tmp_path / "dp")
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, out, dtype)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    d, opt = _make(dev, dtype)
    x0, cond, t, noise = _batch()
    for _ in range(2):
        train_step(d, opt, x0.to(dev), cond.to(dev), 1.0, None, t=t.to(dev), noise=noise.to(dev))
    full = opt.flat.data.cpu()
    p0, p1 = torch.load(f"{out}.0", weights_only=True), torch.load(f"{out}.1", weights_only=True)
    assert torch.equal(p0, p1)
    moved = (full - p0).abs()
    print(f"dp vs full batch ({dtype}): rel {rel(p0, full):.2e}, max abs {moved.max().item():.2e}")
    # Adam moves each element ~lr*sign(g) in the first steps; reduction-order noise (fp32 accumulators in both
    # modes: the bf16 path rounds the same per-sample activations, only the batch sums regroup) can only flip the
    # sign where |g| is at noise level, so compare element-wise against the step scale
    # fp32: < 0.1 % of the entries off by > 0.05 lr, whole vector rel < 1e-5.  bf16: the gradients' noise floor is
    # higher (every stored activation is bf16-rounded, so a regrouped batch sum flips downstream roundings), and the
    # entries whose gradient sits at it move by up to +-lr in either run: measured 0.08-0.11 % of the entries and
    # rel 0.8-1.1e-4 over two runs -> gates 0.5 % and 3e-4 (a wrong reduction moves O(1) of the entries)
    frac_gate, rel_gate = (1e-3, 1e-5) if dtype == torch.float32 else (5e-3, 3e-4)
    assert (moved > 0.05 * 1e-3).double().mean().item() < frac_gate
    assert rel(p0, full) < rel_gate


def test_bench_multirank_gloo_rehearsal():
    """bench.py's N > 1 path -- D.setup, the barrier, the MAX all-reduce of the elapsed time, the rank-0-only
    JSON line and destroy_process_group (reference: train.py:207-221, 1075-1076) -- run as the driver runs it
    (torch.distributed.run, one process per rank), 2 ranks sharing the one GPU over gloo"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--dist-backend", "gloo", "--steps", "2", "--warmup", "2", "--no-cpu-baseline", "--other-configs", "",
           "--batch", "1", "--height", "64", "--width", "96"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and np.isfinite(out["loss"]) and out["steps"] == 2
