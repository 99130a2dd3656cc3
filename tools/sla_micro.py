"""Level-0 sized fused SLA fwd+bwd launches (for rocprofv3 counter passes).
usage: python tools/sla_micro.py [reps] [emit 0|1]"""
import sys

import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import kernels as K  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    emit = (sys.argv[2] != '0') if len(sys.argv) > 2 else True
    Nf, H, W, C = 48, 192, 288, 64
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(Nf, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn_like(x)
    gamma = torch.ones(C, device=dev)
    wqkv = torch.randn(768, C, device=dev) * C ** -0.5
    wout = torch.randn(C, 256, device=dev) * 256 ** -0.5
    bout = torch.zeros(C, device=dev)
    wq = K.conv_pack(wqkv, torch.bfloat16, 768, C, 1, 1, 0, 0)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wq_t = K.conv_pack(wqkv, torch.bfloat16, C, 768, 1, 1, 1, 1)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    dgamma = torch.zeros(C, device=dev)
    for _ in range(reps):
        y, st = K.slaf_fwd(x, gamma, wq, wo, bout, 32 ** -0.5)
        K.slaf_bwd(x, dy, gamma, wq, wq_t, wo_t, st, dgamma, 32 ** -0.5, want_wgrad_inputs=emit)
    torch.cuda.synchronize()
    print("ok", float(y.float().abs().mean()))


if __name__ == "__main__":
    main()
