"""Phase breakdown of twh_bwd_kernel (head-parallel fused temporal backward) from the diagnostic build's
in-kernel stamps.  usage: CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_diag.so python tools/twh_stamps.py [B]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import _lib  # noqa: E402
from cesm_emulator_amd import kernels as K  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    C, F, H, W = 64, 12, 192, 288
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(B * F, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn_like(x)
    gamma = torch.ones(C, device=dev)
    wqkv = torch.randn(768, C, device=dev) * C ** -0.5
    wout = torch.randn(C, 256, device=dev) * 256 ** -0.5
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    bias = K.relpos_fwd(torch.randn(32, 8, device=dev), F)
    rot = K.rope_table(1.0 / (10000 ** (torch.arange(0, 32, 2, device=dev).float() / 32)), F)
    _, mr, lse, _ = K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=True)
    dwq = torch.zeros(768, C, device=dev)
    dgam = torch.zeros(C, device=dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    K.tblock_bwd_dw(x, dy, mr, lse, wqkv, gamma, wo_t, bias, rot, dwq, dgam, None, B, F, 32 ** -0.5)
    e.record()
    torch.cuda.synchronize()
    n = 4096 * 8
    buf = (ctypes.c_ulonglong * n)()
    fn = _lib.lib().cesm_diag_tw_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.float64)
    a = a[a.sum(1) > 0]
    names = ["LN + barrier A", "lse + qkv", "dO", "core (4 px)", "dW GEMM", "dxn + atomics + barrier B",
             "LN bwd + dx", "-"]
    tot = a.sum(1).mean()
    print(f"kernel {s.elapsed_time(e) * 1e3:.0f} us; waves {len(a)}, mean cycles per wave {tot:.3e}")
    for i in range(7):
        print(f"  {names[i]:28s} {a[:, i].mean():.3e}  {100 * a[:, i].mean() / tot:5.1f} %")


if __name__ == "__main__":
    main()
