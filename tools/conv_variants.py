"""Per-level 3x3 conv forward time of the kernel the planner picks (bench shapes, N = 96, bf16); run under
different CESM_CONV3X3_* env settings for an A/B of the halo-conv variants."""
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
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("CESM_CONV3X3")) or "default"
    out = []
    for (H, W, C, C2) in [(192, 288, 64, 0), (96, 144, 128, 0), (48, 72, 256, 0), (24, 36, 512, 0), (192, 288, 64, 64), (96, 144, 128, 128)]:
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        x2 = torch.randn(N, H, W, C2, device=dev).to(torch.bfloat16) if C2 else None
        Co = C if not C2 else C
        w = torch.randn(Co, C + C2, 1, 3, 3, device=dev) * 0.02
        wp = K.conv_pack(w, torch.bfloat16, Co, C + C2, 3, 3, 0, 0)
        v = K.conv_fwd_variant(torch.bfloat16, N, H, W, C, C2, H, W, Co, Co, 3, 3, 1, 1, 1)
        t = timed(lambda: K.conv_fwd(x, x2, wp, None, (H, W, Co, 3, 3, 1, 1, 1)))
        fl = 2 * 9 * (C + C2) * Co * N * H * W
        out.append(f"{H}x{W}x{C}+{C2}->{Co} {v}: {t:.1f} us ({fl / t / 1e6:.0f} TF/s)")
    # level-0 conv with the fused residual (the ResnetBlock skip gradient in the dgrad)
    x = torch.randn(N, 192, 288, 64, device=dev).to(torch.bfloat16)
    r = torch.randn_like(x)
    wp = K.conv_pack(torch.randn(64, 64, 1, 3, 3, device=dev) * 0.02, torch.bfloat16, 64, 64, 3, 3, 0, 0)
    t = timed(lambda: K.conv_fwd(x, None, wp, None, (192, 288, 64, 3, 3, 1, 1, 1), res=r))
    out.append(f"192x288x64 + residual: {t:.1f} us")
    print(f"[{tag}] " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
