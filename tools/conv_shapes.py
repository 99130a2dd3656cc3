"""Log the conv launches of one bench training step (shape, count, FLOP): python tools/conv_shapes.py"""
import collections
import os
import subprocess
import sys

os.environ["CESM_TRACE_CONV"] = "1"
sys.path.insert(0, ".")
import torch  # noqa: E402

from cesm_emulator_amd import kernels as K  # noqa: E402
import bench  # noqa: E402,F401


def main():
    sys.argv = ["bench.py", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
    K.CONV_TRACE.clear()
    bench.main()
    n = len(K.CONV_TRACE) // 2  # warmup + timed step
    c = collections.Counter(K.CONV_TRACE[n:])
    rows = []
    for (kind, Nb, Hi, Wi, Cin, Ho, Wo, Cout, KH, KW, St, Pd, U), k in c.items():
        taps = KH * KW if U == 1 else max(1, KH * KW // (U * U))
        flop = 2.0 * Nb * Ho * Wo * Cout * Cin * taps
        rows.append((flop * k, kind, k, f"N{Nb} {Hi}x{Wi}x{Cin} -> {Ho}x{Wo}x{Cout} k{KH} s{St} p{Pd} u{U}"))
    for f, kind, k, d in sorted(rows, reverse=True):
        print(f"{kind:5s} x{k:2d} {f / 1e9:8.1f} GFLOP  {d}")


if __name__ == "__main__":
    main()
