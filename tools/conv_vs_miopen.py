"""Level-by-level 3x3 conv forward: this library's halo / persistent kernels vs MIOpen (torch conv2d,
channels-last bf16) on the bench shapes (more_blocks, B*F = 96).  usage: python tools/conv_vs_miopen.py"""
import sys

import torch
import torch.nn.functional as Fn

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
    torch.backends.cudnn.benchmark = True
    for (H, W, C) in [(192, 288, 64), (96, 144, 128), (48, 72, 256), (24, 36, 512)]:
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        w = torch.randn(C, C, 1, 3, 3, device=dev) * 0.02
        b = torch.randn(C, device=dev) * 0.1
        wp = K.conv_pack(w, torch.bfloat16, C, C, 3, 3, 0, 0)
        t_ours = timed(lambda: K.conv_fwd(x, None, wp, b, (H, W, C, 3, 3, 1, 1, 1)))
        xt = x.permute(0, 3, 1, 2)  # NCHW view of channels-last memory
        w2 = w[:, :, 0].to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bb = b.to(torch.bfloat16)
        t_mi = timed(lambda: Fn.conv2d(xt, w2, bb, padding=1))
        y_ours = K.conv_fwd(x, None, wp, b, (H, W, C, 3, 3, 1, 1, 1)).float()
        y_mi = Fn.conv2d(xt, w2, bb, padding=1).permute(0, 2, 3, 1).float()
        err = float((y_ours - y_mi).norm() / y_mi.norm())
        fl = 2 * 9 * C * C * N * H * W
        print(f"{H}x{W}x{C}: ours {t_ours:.1f} us ({fl / t_ours / 1e6:.0f} TF/s), MIOpen {t_mi:.1f} us "
              f"({fl / t_mi / 1e6:.0f} TF/s), rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
