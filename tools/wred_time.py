"""HIP-event timing of the 3x3 weight-gradient launches (split-K kernel + conv_wgrad_reduce) at the bench's
four level shapes (B = 8, F = 12, more_blocks): python tools/wred_time.py  (CESM_HIP_LIB picks the library)."""
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
    tag = os.environ.get("CESM_HIP_LIB", "default")
    N = 96
    ref = None
    for (H, W, C) in [(192, 288, 64), (96, 144, 128), (48, 72, 256), (24, 36, 512)]:
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        dw = torch.zeros(C, C, 1, 3, 3, device=dev)
        geom = (H, W, C, 3, 3, 1, 1, 1)
        t = timed(lambda: K.conv_wgrad(x, None, dy, None, dw, geom, False, False, accumulate=False))
        ref = dw.double().norm().item()
        print(f"[{tag}] wgrad3x3 {H}x{W}x{C}: {t:.1f} us  |dW| {ref:.6e}", flush=True)
        del x, dy


if __name__ == "__main__":
    main()
