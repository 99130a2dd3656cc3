"""Generate the SURVEY §8(c) C4 fixtures tests/golden/c4_{baseline,more_blocks}.pt from the CPU oracle.

SELF-GENERATED, NOT REFERENCE-GENERATED: the reference ships no golden vectors and could not be imported
here, so these pin the oracle (oracle/ref_cpu.py) across rounds and give the HIP path fixed
targets.  Per config (baseline ch_mults (1,2,4), more_blocks (1,2,4,8), base_ch 64) and F in {1, 3, 8}, B = 2,
32 x 48 grid, fixed seeds:
  * full tensors: x0, cond, t, noise, x_t, the forward output eps_pred on x_t, the loss;
  * per parameter tensor (params at init, loss gradients without clipping, params after two
    train.py:868-880 fp32 steps = clip_grad_norm_(1.0) + AdamW(lr 2e-4, betas (0.9, 0.999), wd 1e-4)): a
    digest = (fp64 sum, fp64 L2 norm, 32 entries at indices drawn from a generator seeded by the tensor's
    name), because the full 10.3 M / 35.2 M-parameter tensors (x3 states x3 window lengths) do not belong in
    the repository.  digest_index() regenerates the indices.
Run: python tests/golden/make_golden_c4.py   (about a minute on 8 cores)
"""
import os
import sys
import zlib

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ref_cpu as R  # noqa: E402

CONFIGS = {"baseline": (1, 2, 4), "more_blocks": (1, 2, 4, 8)}
FRAMES = (1, 3, 8)
B, H, W = 2, 32, 48
NSAMP = 32


def digest_index(name, numel):
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    if numel <= NSAMP:
        return torch.arange(numel)
    return torch.randint(0, numel, (NSAMP,), generator=g)


def digest(named):
    out = {}
    for name, t in named:
        flat = t.detach().reshape(-1).double()
        out[name] = {"sum": flat.sum().item(), "norm": flat.norm().item(),
                     "vals": flat[digest_index(name, flat.numel())].float().clone()}
    return out


def inputs(F, seed):
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(B, 1, H, W, generator=g)
    cond = torch.randn(B, 1, F, H, W, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    noise = torch.randn(B, 1, H, W, generator=g)
    t2 = torch.randint(0, 1000, (B,), generator=g)
    noise2 = torch.randn(B, 1, H, W, generator=g)
    return x0, cond, t, noise, t2, noise2


def make(mults, F):
    seed = 1000 + 10 * F + len(mults)
    torch.manual_seed(seed)
    u = R.UNet(ch_mults=mults)
    d = R.Diffusion(u)
    x0, cond, t, noise, t2, noise2 = inputs(F, seed + 1)
    rec = {"seed": seed, "x0": x0, "cond": cond, "t": t, "noise": noise, "t2": t2, "noise2": noise2,
           "params0": digest(u.named_parameters())}
    with torch.no_grad():
        x_t, _ = d.q_sample(x0, t, noise)
        rec["x_t"] = x_t
        rec["eps_pred"] = u(x_t, cond, t)
    loss = d.loss(x0, cond, t=t, noise=noise)
    loss.backward()
    rec["loss"] = loss.detach()
    rec["grads"] = digest((n, p.grad) for n, p in u.named_parameters() if p.grad is not None)
    opt = R.make_optimizer(d)
    l1 = R.train_step(d, opt, x0, cond, t=t, noise=noise)
    l2 = R.train_step(d, opt, x0, cond, t=t2, noise=noise2)
    rec["step_losses"] = torch.stack([l1, l2])
    rec["params2"] = digest(u.named_parameters())
    return rec


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for name, mults in CONFIGS.items():
        out = {"mults": torch.tensor(mults), "frames": torch.tensor(FRAMES)}
        for F in FRAMES:
            out[f"F{F}"] = make(mults, F)
            print(name, F, "loss", out[f"F{F}"]["loss"].item(), "steps", out[f"F{F}"]["step_losses"].tolist())
        torch.save(out, os.path.join(HERE, f"c4_{name}.pt"))


if __name__ == "__main__":
    main()
