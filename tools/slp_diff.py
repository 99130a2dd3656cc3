"""How the SLP-packed build's repeated forwards differ (RoPE repeatability investigation):
CESM_HIP_LIB=... python tools/slp_diff.py -> per output, differing elements / rows / frames and the size of the
differences between call 0 and calls 1..3, plus the same for the oracle-free reference: the fp32 evaluation of
the folded forward from the kernel's own saved LN stats is not needed -- only call-to-call differences."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from cesm_emulator_amd import kernels as K  # noqa: E402
from test_gpu_determinism import _temporal_inputs  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, F, H, W, C = 2, 12, 192, 288, 64
    x, dy, gamma, wqkv, wout, bias, rot = _temporal_inputs(dev, B, F, H, W)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    fw = [K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=True) for _ in range(4)]
    torch.cuda.synchronize()
    for k in range(1, 4):
        for a, b, nm in zip(fw[0], fw[k], ("y", "mr", "lse", "o")):
            d = (a.float() - b.float()).abs()
            n = int((d > 0).sum())
            if nm in ("y", "o"):
                rows = d.reshape(B, F, H * W, -1).amax(-1)
                fr = [int((rows[:, f] > 0).sum()) for f in range(F)]
                rel = (d.max() / a.float().abs().max()).item()
                ulps = (d / a.float().abs().clamp_min(1e-30))[d > 0]
                print(f"call {k} {nm}: {n} elements differ, max abs {d.max().item():.3e} (rel to max {rel:.2e}), "
                      f"median rel diff {ulps.median().item() if n else 0:.2e}; differing pixel rows per frame {fr}")
            else:
                print(f"call {k} {nm}: {n} elements differ, max abs {d.max().item():.3e}")


if __name__ == "__main__":
    main()
