"""HIP-event timing of the temporal-attention core (unfused path): MFMA flash kernels (default) vs the VALU
kernels (CESM_NO_TFLASH=1).  usage: python tools/tflash_time.py [F] [H] [W] [B] [reps] [pixel_major]"""
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
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 192
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 288
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    pm = len(sys.argv) > 6 and sys.argv[6] == "1"
    HW = H * W
    dev = torch.device("cuda")
    torch.manual_seed(0)
    qkv = torch.randn(B * F * HW, 768, device=dev).to(torch.bfloat16)
    bias = K.relpos_fwd(torch.randn(32, 8, device=dev), F)
    rot = K.rope_table(1.0 / (10000 ** (torch.arange(0, 32, 2, device=dev).float() / 32)), F)
    st = {}

    def fwd():
        st["o"] = K.tattn_fwd(qkv, bias, rot, B, F, HW, 32 ** -0.5, pixel_major=pm)

    tf = timed(fwd, reps)
    out, lse = st["o"]
    dout = torch.randn_like(out)
    dtable = torch.zeros(32, 8, device=dev)

    def bwd():
        K.tattn_bwd(qkv, out, dout, lse, bias, rot, dtable, B, F, HW, 32 ** -0.5, pixel_major=pm)

    tb = timed(bwd, reps)
    flop = 2 * 2 * F * F * 32 * 8 * HW * B
    kind = "VALU" if os.environ.get("CESM_NO_TFLASH", "0") == "1" else "MFMA"
    kind += " fused" if K.tflash_bwd_variant(F, HW).startswith("tflash_bwd_fused") else " 2-kernel"
    kind += " pm" if pm else ""
    print(f"{kind} F={F} {H}x{W} B={B}: fwd {tf:.1f} us ({flop / tf / 1e6:.1f} TF/s)  bwd {tb:.1f} us "
          f"({2.5 * flop / tb / 1e6:.1f} TF/s)  out mean {float(out.float().abs().mean()):.6f}")


if __name__ == "__main__":
    main()
