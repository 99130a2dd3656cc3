"""HIP-event timing of the Down / Up (4x4 stride-2) convs at the bench shapes (more_blocks, B*F = 96):
forward and dgrad of each level.  A/B: CESM_NO_S2HALO=1 selects the generic implicit GEMM."""
import os
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def timed(fn, reps=10):
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
    tag = "generic" if os.environ.get("CESM_NO_S2HALO") else "halo"
    tot = 0.0
    for (H, W, C) in [(192, 288, 64), (96, 144, 128), (48, 72, 256)]:
        Hl, Wl = H // 2, W // 2
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        xl = torch.randn(N, Hl, Wl, C, device=dev).to(torch.bfloat16)
        w = torch.randn(C, C, 1, 4, 4, device=dev) * 0.02
        wd = K.conv_pack(w, torch.bfloat16, C, C, 4, 4, 0, 0)
        wu = K.conv_pack(w, torch.bfloat16, C, C, 4, 4, 1, 1)
        t_d = timed(lambda: K.conv_fwd(x, None, wd, None, (Hl, Wl, C, 4, 4, 2, 1, 1)))
        t_u = timed(lambda: K.conv_fwd(xl, None, wu, None, (H, W, C, 4, 4, 1, 2, 2)))
        yl = torch.randn(N, Hl, Wl, C, device=dev).to(torch.bfloat16)
        dw = torch.zeros(C, C, 1, 4, 4, device=dev)
        t_w = timed(lambda: K.conv_wgrad(x, None, yl, None, dw, (Hl, Wl, C, 4, 4, 2, 1, 1), 0, 0))
        fl = 2 * 16 * C * C * N * Hl * Wl
        print(f"{tag} {H}x{W}x{C}: wgrad {t_w:.1f} us ({fl / t_w / 1e6:.0f} TF/s)", flush=True)
        tot += t_d + t_u + t_w
        print(f"{tag} {H}x{W}x{C}: down {t_d:.1f} us ({fl / t_d / 1e6:.0f} TF/s), up {t_u:.1f} us "
              f"({fl / t_u / 1e6:.0f} TF/s)", flush=True)
    print(f"{tag} total {tot:.1f} us (per step: x2 for down/up, x2 wgrad)")


if __name__ == "__main__":
    main()
