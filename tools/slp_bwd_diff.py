"""Where an SLP-vectorized build's fused temporal backward (twh_bwd, C = 64, F = 12) differs between identical calls
(RoPE / packed-fp32 repeatability investigation): for a few small shapes (down to one 4-pixel group, i.e.
one block), 6 calls on the same inputs; per output the calls that differ from call 0 and, for dx, the differing
(frame, pixel) voxels, channels per voxel and the size of the differences.

  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_slp.so python tools/slp_bwd_diff.py
"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from cesm_emulator_amd import kernels as K  # noqa: E402
from test_gpu_determinism import _temporal_inputs  # noqa: E402


def run(dev, B, H, W, calls=6):
    F, C = 12, 64
    x, dy, gamma, wqkv, wout, bias, rot = _temporal_inputs(dev, B, F, H, W)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    y, mr, lse, o = K.tblock_fwd_fold(x, gamma, wqkv, wo, bias, rot, B, F, 32 ** -0.5, save_o=True)
    outs = []
    for _ in range(calls):
        dwq, dg, dt = torch.zeros(768, C, device=dev), torch.zeros(C, device=dev), torch.zeros(32, 8, device=dev)
        dx = K.tblock_bwd_dw(x, dy, mr, lse, wqkv, gamma, wo_t, bias, rot, dwq, dg, dt, B, F, 32 ** -0.5)
        outs.append((dx, dwq, dg, dt))
    torch.cuda.synchronize()
    nan = [sum(int((~torch.isfinite(t.float())).sum()) for t in o) for o in outs]
    print(f"== B={B} H={H} W={W} ({B * H * W} pixels, {B * H * W // 4} groups); non-finite per call {nan}")
    for k in range(1, calls):
        line = []
        for a, b, nm in zip(outs[0], outs[k], ("dx", "dWqkv", "dgamma", "dtable")):
            d = (a.float() - b.float()).abs()
            n = int((d > 0).sum())
            line.append(f"{nm} {n}")
            if nm == "dx" and n:
                dv = d.reshape(B, F, H * W, C)
                vox = (dv > 0).any(-1)  # [B, F, HW]
                nvox = int(vox.sum())
                frames = vox.any(2).any(0).nonzero().flatten().tolist()
                pix = vox.any(1).any(0).nonzero().flatten().tolist()
                chans = (dv > 0).sum(-1)[vox].float()
                rel = (d / a.float().abs().clamp_min(1e-30))[d > 0]
                line.append(f"[{nvox} voxels, frames {frames}, pixels {pix[:12]}{'...' if len(pix) > 12 else ''}, "
                            f"channels/voxel {chans.min().item():.0f}-{chans.max().item():.0f}, "
                            f"rel diff median {rel.median().item():.1e} max {rel.max().item():.1e}]")
        print(f"call {k}: " + ", ".join(line), flush=True)


def main():
    dev = torch.device("cuda")
    for (B, H, W) in ((1, 1, 4), (1, 2, 4), (1, 4, 4), (1, 12, 16), (2, 48, 72)):
        run(dev, B, H, W)


if __name__ == "__main__":
    main()
