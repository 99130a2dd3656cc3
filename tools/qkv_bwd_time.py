"""Fused qkv backward (csrc/qkvbwd.hip, dqkv read once) against the two-GEMM path it replaces (1x1 dgrad conv +
wide weight-gradient GEMM), per call at the unfused attention paths' shapes: the decadal window's levels (F = 120,
B = 1) and the F = 12 bench's C >= 256 levels (B = 8).  HIP events on the current stream, median of 10 calls.

  python tools/qkv_bwd_time.py
"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402

SHAPES = [("F120 L0", 192 * 288 * 120, 64), ("F120 L1", 96 * 144 * 120, 128), ("F120 L2", 48 * 72 * 120, 256),
          ("F120 L3", 24 * 36 * 120, 512), ("F12 B8 L2", 48 * 72 * 96, 256), ("F12 B8 L3", 24 * 36 * 96, 512)]


def timeit(fn, n=10):
    ts = []
    for _ in range(n + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[2:])
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    for name, M, C in SHAPES:
        dy = torch.randn(M, 768, device=dev).to(torch.bfloat16)
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        w = torch.randn(768, C, 1, 1, 1, device=dev) * C ** -0.5
        wt = K.conv_pack(w, torch.bfloat16, C, 768, 1, 1, 1, 1)
        dw = torch.zeros(768, C, device=dev)
        dw5 = dw.view(768, C, 1, 1, 1)
        t_new = timeit(lambda: K.qkv_bwd(dy, x, wt, dw))
        t_dg = timeit(lambda: K.conv_fwd(dy.view(1, 1, M, 768), None, wt, None, (1, M, C, 1, 1, 1, 0, 1)))
        t_wg = timeit(lambda: K.conv_wgrad(x.view(1, 1, M, C), None, dy.view(1, 1, M, 768), None, dw5,
                                           (1, M, 768, 1, 1, 1, 0, 1), 0, 0))
        gb = M * (768 * 2 + 2 * C * 2) / 1e9  # algorithmic bytes of the fused pass
        print(f"{name:10s} M={M:8d} C={C:3d}: fused {t_new:8.1f} us ({gb / t_new * 1e6 / 1e3:5.2f} TB/s alg.) | "
              f"dgrad {t_dg:8.1f} + wgrad {t_wg:8.1f} = {t_dg + t_wg:8.1f} us | x{(t_dg + t_wg) / t_new:.2f}",
              flush=True)
        del dy, x


if __name__ == "__main__":
    main()
