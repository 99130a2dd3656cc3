"""HIP-event time of the bench's wide weight-gradient GEMMs (dW = dY^T X over the pixels) -- wgrad_wide_kernel through
cesm_conv_wgrad -- next to torch.mm on the same operands (the ROCm BLAS path) as an achievable-rate reference for this
GEMM shape (not used by the product).  usage: python tools/wgrad_vs_blas.py"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from cesm_emulator_amd import kernels as K  # noqa: E402
from tblock_time import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for (name, H, W, C, N) in (("L2 qkv", 48, 72, 256, 768), ("L3 qkv", 24, 36, 512, 768), ("L1 qkv", 96, 144, 128, 768),
                               ("L2 out", 48, 72, 256, 256), ("L0 out", 192, 288, 256, 64)):
        Nb = 96
        M = Nb * H * W
        x = torch.randn(Nb, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(Nb, H, W, N, device=dev).to(torch.bfloat16)
        dw = torch.zeros(N, C, device=dev)
        t_k = timed(lambda: K.conv_wgrad(x, None, dy, None, dw, (H, W, N, 1, 1, 1, 0, 1), 0, 0, accumulate=False), 10)
        a, b = dy.view(M, N), x.view(M, C)
        t_b = timed(lambda: torch.mm(a.t(), b), 10)
        ref = (a.float().t() @ b.float())
        rel = ((dw - ref).norm() / ref.norm()).item()
        fl = 2.0 * M * N * C
        print(f"{name}: M={M} N={N} K={C}: wgrad_wide {t_k:.1f} us ({fl / t_k / 1e6:.0f} TF/s) | torch.mm bf16 {t_b:.1f} us "
              f"({fl / t_b / 1e6:.0f} TF/s) | rel {rel:.1e}", flush=True)


if __name__ == "__main__":
    main()
