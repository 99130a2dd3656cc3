"""Do the fused temporal kernels read registers or LDS they have not written?  Before each call the diagnostic
polluters (tools/diag/libvgpr_pollute.so: every LDS word of each CU, then every VGPR and AGPR of 1 wave per SIMD x
many waves, set to a 32-bit pattern) run on the same stream; the call's outputs must not depend on the pattern.  Patterns: quiet NaN, 0, 1.0f, and 0x7f7f7f7f
(3.4e38 in fp32, a large finite bf16 pair).  For each shape: the outputs of twh_bwd (tblock_bwd_dw) and of the folded
forward after each pattern, compared with the first pattern's, and non-finite counts.

  [CESM_HIP_LIB=...] python tools/vgpr_pollute_check.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from cesm_emulator_amd import kernels as K  # noqa: E402
from test_gpu_determinism import _temporal_inputs  # noqa: E402

POL = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag", "libvgpr_pollute.so"))
POL.vgpr_pollute.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.c_void_p]
POL.lds_pollute.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.c_void_p]
PATTERNS = {"nan": 0x7FC07FC0, "zero": 0, "one": 0x3F800000, "big": 0x7F7F7F7F}


def pollute(bits):
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert POL.lds_pollute(bits, 2048, st) == 0 and POL.vgpr_pollute(bits, 8192, st) == 0, "polluter launch failed"


def main():
    dev = torch.device("cuda")
    F, C = 12, 64
    for (B, H, W) in ((1, 1, 4), (1, 1, 8), (1, 3, 4), (1, 4, 4), (1, 5, 4), (1, 12, 16), (2, 48, 72)):
        x, dy, gamma, wqkv, wout, bias, rot = _temporal_inputs(dev, B, F, H, W)
        wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
        wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
        res = {}
        for name, bits in PATTERNS.items():
            torch.cuda.synchronize()
            pollute(bits)
            y, mr, lse, o = K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=True)
            dwq, dg, dt = torch.zeros(768, C, device=dev), torch.zeros(C, device=dev), torch.zeros(32, 8, device=dev)
            torch.cuda.synchronize()
            pollute(bits)
            dx = K.tblock_bwd_dw(x, dy, mr, lse, wqkv, gamma, wo_t, bias, rot, dwq, dg, dt, B, F, 32 ** -0.5)
            torch.cuda.synchronize()
            res[name] = (y, lse, dx, dwq, dg, dt)
        names = ("y", "lse", "dx", "dWqkv", "dgamma", "dtable")
        base = res["nan"]
        line = [f"B={B} H={H} W={W}:"]
        for name, outs in res.items():
            nf = sum(int((~torch.isfinite(t.float())).sum()) for t in outs)
            diff = [f"{nm} {int((a != b).sum())}" for a, b, nm in zip(base, outs, names) if not torch.equal(a, b)]
            line.append(f"[{name}: non-finite {nf}; vs nan: {', '.join(diff) if diff else 'identical'}]")
        print(" ".join(line), flush=True)


if __name__ == "__main__":
    main()
