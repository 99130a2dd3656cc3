"""Large-batch index-width check at full size (size-independent property): the bf16 loss and gradients
of a batch of B samples must equal the mean over its two halves (per-sample norms, mean loss), so any
32-bit offset overflow that only appears at B*F*H*W*768 > 2^31 elements shows up as a mismatch.
usage: python tools/batch_check.py [B] [F]"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd.model import Diffusion  # noqa: E402
from cesm_emulator_amd.train import build_model_from_config  # noqa: E402
import json  # noqa: E402


def grads(diff, x0, cond, t, noise):
    for p in diff.parameters():
        p.grad = None
    loss = diff.loss(x0, cond, t=t, noise=noise)
    loss.backward()
    return float(loss), {n: p.grad.detach().float().clone() for n, p in diff.named_parameters() if p.grad is not None}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    H, W = 192, 288
    dev = torch.device("cuda")
    cfg = json.load(open("config/more_blocks"))
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    x0 = torch.randn(B, 1, H, W, device=dev, generator=g)
    cond = torch.randn(B, 1, F, H, W, device=dev, generator=g)
    noise = torch.randn(B, 1, H, W, device=dev, generator=g)
    t = torch.randint(0, 1000, (B,), device=dev, generator=g)
    h = B // 2
    lf, gf = grads(diff, x0, cond, t, noise)
    l1, g1 = grads(diff, x0[:h], cond[:h], t[:h], noise[:h])
    l2, g2 = grads(diff, x0[h:], cond[h:], t[h:], noise[h:])
    print(f"peak mem {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB")
    lm = 0.5 * (l1 + l2)
    print(f"loss full {lf:.6f} halves-mean {lm:.6f} rel {abs(lf - lm) / abs(lm):.2e}")
    worst = (0.0, "")
    for n in gf:
        ref = 0.5 * (g1[n] + g2[n])
        e = float((gf[n] - ref).norm() / (ref.norm() + 1e-30))
        if e > worst[0]:
            worst = (e, n)
    print(f"worst grad rel err {worst[0]:.2e} ({worst[1]})")
    ok = abs(lf - lm) / abs(lm) < 1e-2 and worst[0] < 5e-2
    print("OK" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
