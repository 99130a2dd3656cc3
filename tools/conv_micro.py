"""The bench's dominant kernel in isolation: level-0 3x3 conv 64->64 (B=4, F=12, 192x288, bf16),
plus a known-size device copy used to calibrate the FETCH_SIZE / WRITE_SIZE counters
(tools/traffic.py).

usage: python tools/conv_micro.py [reps] [levels]      levels: comma list of U-Net levels (default 0)
       (level l: 64*2^l channels at 192/2^l x 288/2^l; level 0 is the one tools/traffic.py reads)"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def run_level(lvl, reps, dev):
    Nb, H, W, C = 48, 192 >> lvl, 288 >> lvl, 64 << lvl
    torch.manual_seed(0)
    x = torch.randn(Nb, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5
    wp = K.conv_pack(w, torch.bfloat16, C, C, 3, 3, 0, 0)
    b = torch.zeros(C, device=dev)
    geom = (H, W, C, 3, 3, 1, 1, 1)
    for _ in range(2):
        y = K.conv_fwd(x, None, wp, b, geom)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        y = K.conv_fwd(x, None, wp, b, geom)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    flop = 2.0 * Nb * H * W * C * C * 9
    print(f"conv3x3 {C}->{C} Nb={Nb} {H}x{W}: {us:.1f} us  {flop / us / 1e6:.1f} TFLOP/s  "
          f"copy_bytes={x.nbytes}  y={float(y.float().abs().mean()):.4f}", flush=True)
    return x


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    levels = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    dev = torch.device("cuda")
    x = None
    for lvl in levels:
        xl = run_level(lvl, reps, dev)
        if lvl == 0:
            x = xl
    if x is not None:
        # calibration, the LAST dispatch of the run: one elementwise pass reading exactly x.nbytes and
        # writing x.nbytes
        z = torch.empty_like(x)
        torch.neg(x, out=z)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
