"""HIP-event time of the level-0 head-parallel temporal backward (tblock_bwd_dw, C = 64, F = 12) with and without the O
emission (round 6), and of the folded forward with and without its O write.  usage: python tools/twh_o_time.py [B] [reps]"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from cesm_emulator_amd import kernels as K  # noqa: E402
from tblock_time import timed  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
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
    y, mr, lse, o = K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=True)
    dwq = torch.zeros(768, C, device=dev)
    dg = torch.zeros(C, device=dev)
    dt = torch.zeros(32, 8, device=dev)
    res = {}
    for emit in (False, True, False, True):
        res.setdefault(emit, []).append(timed(
            lambda: K.tblock_bwd_dw(x, dy, mr, lse, wqkv, gamma, wo_t, bias, rot, dwq, dg, dt, B, F, 32 ** -0.5,
                                    emit_o=emit), reps))
    for save_o in (True, False, True, False):
        res.setdefault(("fwd", save_o), []).append(timed(
            lambda: K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=save_o), reps))
    _, ob = K.tblock_bwd_dw(x, dy, mr, lse, wqkv, gamma, wo_t, bias, rot, None, None, None, B, F, 32 ** -0.5,
                            emit_o=True)
    d = (ob.float() - o.float()).norm() / o.float().norm()
    print(f"B={B}: bwd without O {min(res[False]):.1f} us, with O {min(res[True]):.1f} us; fwd with O "
          f"{min(res[('fwd', True)]):.1f} us, without {min(res[('fwd', False)]):.1f} us; net per block "
          f"{min(res[('fwd', True)]) - min(res[('fwd', False)]) - (min(res[True]) - min(res[False])):.1f} us saved; "
          f"O(bwd) vs O(fwd) rel {d.item():.2e}", flush=True)


if __name__ == "__main__":
    main()
