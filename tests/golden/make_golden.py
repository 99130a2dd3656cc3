"""Generate tests/golden/oracle_small.pt from the CPU oracle (self-generated fixture: the reference
ships no golden vectors and could not be imported here — SURVEY.md §8(c) C1/C4).

Contents: the seed of a small UNet (base_ch 64, ch_mults (1,2)) plus per-tensor weight sums (the
weights themselves are regenerated from the seed), inputs (x0, cond, t, noise), the forward output
on x_t, the loss, and every parameter-gradient L2 norm.
Run: python tests/golden/make_golden.py
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ref_cpu as R  # noqa: E402


def main():
    torch.manual_seed(0)
    u = R.UNet(base_ch=64, ch_mults=(1, 2))
    d = R.Diffusion(u)
    g = torch.Generator().manual_seed(123)
    x0 = torch.randn(2, 1, 16, 24, generator=g)
    cond = torch.randn(2, 1, 3, 16, 24, generator=g)
    t = torch.tensor([5, 871])
    noise = torch.randn(2, 1, 16, 24, generator=g)
    loss = d.loss(x0, cond, t=t, noise=noise)
    loss.backward()
    with torch.no_grad():
        x_t, _ = d.q_sample(x0, t, noise)
        eps = u(x_t, cond, t)
    out = {"seed": torch.tensor(0), "weight_sums": {n: v.double().sum().item() for n, v in u.state_dict().items()},
           "x0": x0, "cond": cond, "t": t, "noise": noise, "eps_pred": eps,
           "loss": loss.detach(),
           "grad_norms": {n: p.grad.norm().item() for n, p in u.named_parameters() if p.grad is not None}}
    torch.save(out, os.path.join(HERE, "oracle_small.pt"))
    print("loss", loss.item())


if __name__ == "__main__":
    main()
