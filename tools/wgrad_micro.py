"""3x3 weight-gradient launches at U-Net level l (for rocprofv3 counter passes / timing).
usage: python tools/wgrad_micro.py [reps] [levels]"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    levels = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 3]
    dev = torch.device("cuda")
    for lvl in levels:
        Nb, H, W, C = 96, 192 >> lvl, 288 >> lvl, 64 << lvl
        torch.manual_seed(0)
        x = torch.randn(Nb, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(Nb, H, W, C, device=dev).to(torch.bfloat16)
        dw = torch.zeros(C, C, 1, 3, 3, device=dev)
        geom = (H, W, C, 3, 3, 1, 1, 1)
        for _ in range(2):
            K.conv_wgrad(x, None, dy, None, dw, geom, 0, 0)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            K.conv_wgrad(x, None, dy, None, dw, geom, 0, 0)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        flop = 2.0 * Nb * H * W * C * C * 9
        v = K.conv_wgrad_variant(torch.bfloat16, Nb, H, W, C, 0, H, W, C, C, 3, 3, 1, 1, 1, False) \
            if hasattr(K, "conv_wgrad_variant") else "?"
        print(f"wgrad3x3 level {lvl} {C}->{C} {v}: {us:.1f} us {flop / us / 1e6:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
