"""HIP-event timing of the wide-tile 1x1 weight gradients at the level-0 / level-1 bench shapes (A/B via
CESM_HIP_LIB)."""
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
    out = []
    for (H, W, Cx, Cy, bias) in [(192, 288, 256, 64, False), (192, 288, 256, 64, True), (96, 144, 128, 768, False),
                                 (96, 144, 256, 128, True)]:
        x = torch.randn(N, H, W, Cx, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, H, W, Cy, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Cy, Cx, 1, 1, 1, device=dev)
        db = torch.zeros(Cy, device=dev) if bias else None
        t = timed(lambda: K.conv_wgrad(x, None, dy, None, dw, (H, W, Cy, 1, 1, 1, 0, 1), 0, 0, db=db))
        gb = N * H * W * (Cx + Cy) * 2 / 1e9
        out.append(f"{H}x{W} {Cx}->{Cy}{' +b' if bias else ''}: {t:.0f} us ({gb / t * 1e6:.0f} GB/s)")
    print(f"[{os.environ.get('CESM_HIP_LIB', 'default')}] " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
