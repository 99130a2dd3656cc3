"""HIP-event timing of the 1x1 convs (gemm1x1_kernel) at bench shapes (more_blocks, B*F = 96): the unfused
attention projections of levels 2-3 and their data gradients, and level-0/1 res_convs.
usage: [CESM_HIP_LIB=...] [G1_SHAPES=f120] python tools/gemm_time.py
G1_SHAPES=f120: the long-window leg (B = 1, F = 120): each level's unfused temporal-block projections
(to_qkv C -> 768, to_out 256 -> C) and their data gradients (768 -> C, C -> 256)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda")
    N = 96
    out, tot = [], 0.0
    shapes = [(48, 72, 256, 0, 768), (48, 72, 768, 0, 256), (48, 72, 256, 0, 256),
                                 (24, 36, 512, 0, 768), (24, 36, 768, 0, 512), (24, 36, 256, 0, 512),
                                 (192, 288, 64, 64, 64), (96, 144, 128, 128, 128)]
    if os.environ.get("G1_SHAPES") == "f120":
        N = 120
        shapes = [(H, W, a, 0, b) for (H, W, C) in [(192, 288, 64), (96, 144, 128), (48, 72, 256), (24, 36, 512)]
                  for (a, b) in [(C, 768), (256, C), (768, C), (C, 256)]]
    for (H, W, C1, C2, Cout) in shapes:
        x1 = torch.randn(N, H, W, C1, device=dev).to(torch.bfloat16)
        x2 = torch.randn(N, H, W, C2, device=dev).to(torch.bfloat16) if C2 else None
        w = torch.randn(Cout, C1 + C2, 1, 1, 1, device=dev) * 0.05
        wp = K.conv_pack(w, torch.bfloat16, Cout, C1 + C2, 1, 1, 0, 0)
        b = torch.randn(Cout, device=dev)
        v = K.conv_fwd_variant(torch.bfloat16, N, H, W, C1, C2, H, W, Cout, Cout, 1, 1, 1, 0, 1)
        t = timed(lambda: K.conv_fwd(x1, x2, wp, b, (H, W, Cout, 1, 1, 1, 0, 1)))
        tot += t
        fl = 2.0 * N * H * W * (C1 + C2) * Cout
        by = N * H * W * (C1 + C2 + Cout) * 2
        out.append(f"{H}x{W} {C1}+{C2}->{Cout} {v}: {t:.1f} us ({fl / t / 1e6:.0f} TF/s, {by / t / 1e3:.0f} GB/s)")
    print("\n".join(out) + f"\ntotal {tot:.1f} us", flush=True)


if __name__ == "__main__":
    main()
