"""HIP-event timing of the GroupNorm passes at the level-0 bench shape (B = 8, F = 12, 192x288, C = 64) and
level 1 (96x144, C = 128): stats, apply (with / without residual), backward (reduce + apply); effective GB/s.
GN_SHAPES=f120: the long-window leg instead (B = 1, F = 120, levels 0 and 1)."""
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
    B, F, G = 8, 12, 8
    if os.environ.get("GN_SHAPES") == "f120":
        B, F = 1, 120
    tag = os.environ.get("CESM_HIP_LIB", "default") + f" B={B} F={F}"
    for (H, W, C) in [(192, 288, 64), (96, 144, 128)]:
        y = torch.randn(B * F, H, W, C, device=dev).to(torch.bfloat16)
        res = torch.randn_like(y)
        dz = torch.randn_like(y)
        gamma = torch.rand(C, device=dev) + 0.5
        beta = torch.randn(C, device=dev) * 0.1
        ss = torch.randn(B, 2 * C, device=dev) * 0.1
        dg, db, dbias = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        st = K.gn_stats(y, B, G)
        nb = y.numel() * 2
        t_s = timed(lambda: K.gn_stats(y, B, G))
        t_a = timed(lambda: K.gn_apply(y, st, gamma, beta, ss, None, B, G))
        t_ar = timed(lambda: K.gn_apply(y, st, gamma, beta, None, res, B, G))
        t_b = timed(lambda: K.gn_bwd(dz, y, st, gamma, beta, ss, dg, db, B, G, True, dbias=dbias))
        print(f"[{tag}] {H}x{W}x{C}: stats {t_s:.0f} us ({nb / t_s / 1e3:.0f} GB/s), apply {t_a:.0f} us "
              f"({2 * nb / t_a / 1e3:.0f}), apply+res {t_ar:.0f} us ({3 * nb / t_ar / 1e3:.0f}), bwd {t_b:.0f} us "
              f"({5 * nb / t_b / 1e3:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
