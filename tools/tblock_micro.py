"""Level-0 sized fused temporal-block fwd+bwd launches (for rocprofv3 counter passes).
usage: python tools/tblock_micro.py [C] [reps] [emit 0|1]"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    emit = (sys.argv[3] != '0') if len(sys.argv) > 3 else True
    B, F = 4, 12
    H, W = {64: (192, 288), 128: (96, 144), 256: (48, 72), 512: (24, 36)}[C]
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
    for _ in range(reps):
        y, mr, lse, _ = K.tblock_fwd(x, gamma, wq, wo, bias, rot, B, F, 32 ** -0.5)
        K.tblock_bwd(x, dy, gamma, mr, lse, wq, wq_t, wo_t, bias, rot, dgamma, dtable, B, F, 32 ** -0.5,
                      want_wgrad_inputs=emit)
    torch.cuda.synchronize()
    print("ok", float(y.float().abs().mean()))


if __name__ == "__main__":
    main()
