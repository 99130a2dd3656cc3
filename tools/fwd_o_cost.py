"""Cost of the O write in the fused temporal forwards: HIP-event time of tblock_fwd_fold (C = 64,
level 0) and tblock_fwd (C = 128, level 1) with and without save_o, and of the to_out weight-gradient GEMM that reads
the saved O.  usage: python tools/fwd_o_cost.py [B] [reps]"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402
from tblock_time import timed  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    F = 12
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for C, (H, W) in ((64, (192, 288)), (128, (96, 144))):
        x = torch.randn(B * F, H, W, C, device=dev).to(torch.bfloat16)
        gamma = torch.ones(C, device=dev)
        wqkv = torch.randn(768, C, device=dev) * C ** -0.5
        wout = torch.randn(C, 256, device=dev) * 256 ** -0.5
        wq = K.conv_pack(wqkv, torch.bfloat16, 768, C, 1, 1, 0, 0)
        wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
        bias = K.relpos_fwd(torch.randn(32, 8, device=dev), F)
        rot = K.rope_table(1.0 / (10000 ** (torch.arange(0, 32, 2, device=dev).float() / 32)), F)
        res = {}
        for save_o in (True, False, True, False):
            if C == 64:
                fn = lambda: K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=save_o)  # noqa
            else:
                fn = lambda: K.tblock_fwd(x, gamma, wq, wo, bias, rot, B, F, 32 ** -0.5, save_o=save_o)  # noqa
            res.setdefault(save_o, []).append(timed(fn, reps))
        o = torch.randn(B * F, H, W, 256, device=dev).to(torch.bfloat16)
        dy = torch.randn_like(x)
        dwo = torch.zeros(C, 256, device=dev)
        tw = timed(lambda: K.conv_wgrad(o, None, dy, None, dwo, (H, W, C, 1, 1, 1, 0, 1), 0, 0), reps)
        print(f"C={C} B={B}: fwd with O {min(res[True]):.1f} us, without O {min(res[False]):.1f} us "
              f"(O write {min(res[True]) - min(res[False]):.1f} us); to_out wgrad from O {tw:.1f} us", flush=True)


if __name__ == "__main__":
    main()
