"""HIP-event timing of the level-0 fused temporal / SLA block kernels (A/B of variant libraries:
CESM_HIP_LIB=... python tools/tblock_time.py [C] [reps])."""
import os
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def timed(fn, reps):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    B, F = (int(sys.argv[3]) if len(sys.argv) > 3 else 8), 12
    H, W = {64: (192, 288), 128: (96, 144)}[C]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(B * F, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn_like(x)
    gamma = torch.ones(C, device=dev)
    wqkv = torch.randn(768, C, device=dev) * C ** -0.5
    wout = torch.randn(C, 256, device=dev) * 256 ** -0.5
    wq = K.conv_pack(wqkv, torch.bfloat16, 768, C, 1, 1, 0, 0)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wq_t = K.conv_pack(wqkv, torch.bfloat16, C, 768, 1, 1, 1, 1)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    bias = K.relpos_fwd(torch.randn(32, 8, device=dev), F)
    rot = K.rope_table(1.0 / (10000 ** (torch.arange(0, 32, 2, device=dev).float() / 32)), F)
    dgamma = torch.zeros(C, device=dev)
    dtable = torch.zeros(32, 8, device=dev)
    st = {}

    def fwd():
        st["r"] = K.tblock_fwd(x, gamma, wq, wo, bias, rot, B, F, 32 ** -0.5, save_o=True)

    tf = timed(fwd, reps)
    y, mr, lse, o = st["r"]

    def bwd():
        K.tblock_bwd(x, dy, gamma, mr, lse, wq, wq_t, wo_t, bias, rot, dgamma, dtable, B, F, 32 ** -0.5,
                     want_wgrad_inputs=os.environ.get("TW_NOEMIT", "0") == "0", emit_o=False)

    tb = timed(bwd, reps)
    # the old path's to_qkv weight gradient from the emitted dqkv / xn (what the dw kernel replaces)
    st["b"] = K.tblock_bwd(x, dy, gamma, mr, lse, wq, wq_t, wo_t, bias, rot, dgamma, dtable, B, F, 32 ** -0.5,
                           want_wgrad_inputs=True, emit_o=False)
    dwq = torch.zeros(768, C, device=dev)

    def qwgrad():
        _, dqkv, _, xn = st["b"]
        K.conv_wgrad(xn, None, dqkv, None, dwq, (H, W, 768, 1, 1, 1, 0, 1), 0, 0)

    tqw = timed(qwgrad, reps)
    tdw = float("nan")
    if C == 64 and K.tblock_bwd_dw_supported(B, F, H * W, C):
        wo_pack = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
        yf, mrf, lsef, of = K.tblock_fwd_fold(x, gamma, wqkv, wo_pack, bias, rot, B, F, 32 ** -0.5, save_o=True)

        def bwd_dw():
            K.tblock_bwd_dw(x, dy, mrf, lsef, wqkv, gamma, wo_t, bias, rot, dwq, dgamma, dtable, B, F, 32 ** -0.5)

        tdw = timed(bwd_dw, reps)
        # round 5: the in-kernel to_out weight gradient (no O from the forward) vs the O path's forward + wide wgrad
        dwo = torch.zeros(C, 256, device=dev)

        def bwd_dwo():
            K.tblock_bwd_dw(x, dy, mrf, lsef, wqkv, gamma, wo_t, bias, rot, dwq, dgamma, dtable, B, F, 32 ** -0.5,
                            dwout=dwo)

        tdwo = timed(bwd_dwo, reps)
        tfo = timed(lambda: K.tblock_fwd_fold(x, gamma, wqkv, wo_pack, bias, rot, B, F, 32 ** -0.5, save_o=True), reps)
        tfn = timed(lambda: K.tblock_fwd_fold(x, gamma, wqkv, wo_pack, bias, rot, B, F, 32 ** -0.5, save_o=False), reps)
        two = timed(lambda: K.conv_wgrad(of, None, dy, None, dwo, (H, W, C, 1, 1, 1, 0, 1), 0, 0), reps)
        print(f"fold: fwd with O {tfo:.1f} us, without O {tfn:.1f} us; bwd_dw {tdw:.1f} us + O^T dy wgrad {two:.1f} us "
              f"= O path {tfo + tdw + two:.1f} us; bwd_dw with in-kernel dW_out {tdwo:.1f} us = {tfn + tdwo:.1f} us",
              flush=True)
    bout = torch.randn(C, device=dev) * 0.1

    def sfwd():
        st["s"] = K.slaf_fwd(x, gamma, wq, wo, bout, 32 ** -0.5, save_o=True)

    sf = timed(sfwd, reps)
    ys, sst = st["s"]

    def sbwd():
        K.slaf_bwd(x, dy, gamma, wq, wq_t, wo_t, sst, dgamma, 32 ** -0.5,
                   want_wgrad_inputs=os.environ.get("TW_NOEMIT", "0") == "0")

    sb = timed(sbwd, reps)
    # the old SLA path's to_qkv weight gradient, and the in-kernel-dW backward (C = 64)
    st["sb"] = K.slaf_bwd(x, dy, gamma, wq, wq_t, wo_t, sst, dgamma, 32 ** -0.5, want_wgrad_inputs=True)

    def sqwgrad():
        _, dqkv, _, xn = st["sb"]
        K.conv_wgrad(xn, None, dqkv, None, dwq, (H, W, 768, 1, 1, 1, 0, 1), 0, 0)

    tsq = timed(sqwgrad, reps)
    tsdw = float("nan")
    if K.slaf_bwd_dw_supported(B * F, H * W, C):
        ones = torch.ones(C, device=dev)
        wqf = K.pack_scaled(wqkv, gamma)
        _, sstf = K.slaf_fwd(x, ones, wqf, wo, bout, 32 ** -0.5, save_o=True)

        def sbwd_dw():
            K.slaf_bwd_dw(x, dy, ones, wqf, wqkv, gamma, wo_t, sstf, dwq, dgamma, 32 ** -0.5)

        tsdw = timed(sbwd_dw, reps)
    lib = os.environ.get("CESM_HIP_LIB", "default") + (" noemit" if os.environ.get("TW_NOEMIT", "0") != "0" else "")
    print(f"{lib}: C={C} tw_fwd {tf:.1f} us  tw_bwd {tb:.1f} us (+ qkv wgrad {tqw:.1f} us)  tw_bwd_dw {tdw:.1f} us  "
          f"sla_fwd {sf:.1f} us  sla_bwd {sb:.1f} us (+ qkv wgrad {tsq:.1f} us)  sla_bwd_dw {tsdw:.1f} us  "
          f"y {float(y.float().abs().mean()):.6f} ys {float(ys.float().abs().mean()):.6f}")


if __name__ == "__main__":
    main()
