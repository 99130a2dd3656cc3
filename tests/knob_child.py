"""Cases for tests/test_gpu_knobs.py (and the polluter runs of tests/test_gpu_stale_state.py), computed in a process whose environment selects a kernel variant.

The library reads its dispatch knobs (CESM_CONV_WS) once per process (common.h getenv_flag caches
the first lookup), so a knob-on result comes from a child process started with the knob set before any GPU call:

  CESM_CONV_WS=1 python tests/knob_child.py <case> <out.pt>

writes {"variant": <kernel name the dispatch picked>, <tensor name>: <CPU tensor>, ...}; the parent computes the
same case in its own (default) environment with compute() and compares.  Inputs are seeded on the CPU, so both
processes see the same bits.  Not a test module (no test_ prefix): it runs only as that child.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

from cesm_emulator_amd import kernels as K  # noqa: E402

BF = torch.bfloat16

# conv3x3ws shapes that are opt-in (CESM_CONV_WS=1): 128 / 256 channels (ncob > 1: per-step weight DMA, the
# ws_decode co-block order, GN slots at cb * 16), concat inputs (the x2 chunk source), Cout != Cin.
# (C1, C2, Cout, H, W, B, Fr): 24 x 96 and 16 x 288 are covered exactly by 8 x 32 tiles (ws utilisation 1.0)
CONV_CASES = {
    "c128": (128, 0, 128, 24, 96, 2, 2),
    "c64x64": (64, 64, 64, 24, 96, 2, 2),
    "c64to128": (64, 0, 128, 16, 288, 1, 2),
    "c128x64to64": (128, 64, 64, 24, 96, 1, 3),
    "c256": (256, 0, 256, 24, 96, 1, 2),
}
# long-window core (F, HW, B): F = 120 (config 4), and frame counts with a partial 16-frame tile
TF_CASES = {"f120": (120, 77, 2), "f33": (33, 300, 1), "f17": (17, 40, 3), "f12": (12, 300, 2)}


def conv_case(name, dev):
    C1, C2, Cout, H, W, B, Fr = CONV_CASES[name]
    Nb = B * Fr
    g = torch.Generator().manual_seed(C1 * 7 + C2 * 3 + Cout + H + W)
    x1 = (torch.randn(Nb, H, W, C1, generator=g) + 0.3).to(dev, BF)
    x2 = torch.randn(Nb, H, W, C2, generator=g).to(dev, BF) if C2 else None
    w = torch.randn(Cout, C1 + C2, 1, 3, 3, generator=g) * (C1 + C2) ** -0.5 / 3
    bias = torch.randn(Cout, generator=g) * 0.5
    res = torch.randn(Nb, H, W, Cout, generator=g).to(dev, BF)
    wp = K.conv_pack(w.to(dev), BF, Cout, C1 + C2, 3, 3, 0, 0)
    bias = bias.to(dev)
    geom = (H, W, Cout, 3, 3, 1, 1, 1)
    out = {"variant": K.conv_fwd_variant(BF, Nb, H, W, C1, C2, H, W, Cout, Cout, 3, 3, 1, 1, 1)}
    out["y"] = K.conv_fwd(x1, x2, wp, bias, geom)
    out["y_res"] = K.conv_fwd(x1, x2, wp, bias, geom, res=res)
    nslot = K.conv_gn_nslot(x1, x2, geom, B)
    y_gn, part = K.conv_fwd_gn(x1, x2, wp, bias, geom, B, nslot)
    out["y_gn"] = y_gn
    out["gn_stats"] = K.gn_stats_part(part, y_gn.numel() // (Cout * B), 8)
    out["gn_stats_ref"] = K.gn_stats(y_gn, B, 8)  # the separate statistics pass over the stored y
    torch.cuda.synchronize()
    return {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in out.items()}


def tf_case(name, dev):
    F, HW, B = TF_CASES[name]
    g = torch.Generator().manual_seed(F * 100 + HW)
    scale = 32 ** -0.5
    freqs = 1.0 / (10000 ** (torch.arange(0, 32, 2).float() / 32))
    bias = K.relpos_fwd(torch.randn(32, 8, generator=g).to(dev), F)
    rot = K.rope_table(freqs.to(dev), F)
    qkv = torch.randn(B * F * HW, 768, generator=g).to(dev, BF)
    dy = torch.randn(B * F * HW, 256, generator=g).to(dev, BF)
    to_pm = lambda t: t.view(B, F, HW, -1).transpose(1, 2).reshape(B * F * HW, -1).contiguous()  # noqa: E731
    from_pm = lambda t: t.view(B, HW, F, -1).transpose(1, 2).reshape(B * F * HW, -1)  # noqa: E731
    out = {"variant": K.tflash_bwd_variant(F, HW)}
    o, lse = K.tattn_fwd(qkv, bias, rot, B, F, HW, scale)
    dt = torch.zeros(32, 8, device=dev)
    out["dqkv"] = K.tattn_bwd(qkv, o, dy, lse, bias, rot, dt, B, F, HW, scale)
    out["dtable"] = dt
    if F <= 16:  # pixel-major qkv rows are a long-window layout (F > 16)
        torch.cuda.synchronize()
        return {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in out.items()}
    # the output (and so dy) is frame-major for either qkv layout; dq / dk / dv come back in the qkv's order
    o_pm, lse_pm = K.tattn_fwd(to_pm(qkv), bias, rot, B, F, HW, scale, pixel_major=True)
    dt_pm = torch.zeros(32, 8, device=dev)
    out["dqkv_pm"] = from_pm(K.tattn_bwd(to_pm(qkv), o_pm, dy, lse_pm, bias, rot, dt_pm, B, F, HW, scale,
                                         pixel_major=True))
    out["dtable_pm"] = dt_pm
    torch.cuda.synchronize()
    return {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in out.items()}


def train_step_case(dev):
    """one bf16 training step of more_blocks (64 x 96, F = 12, B = 2): loss, every parameter gradient and the peak
    allocated memory of the step (for CESM_WGRAD_STREAM=1 against the default)"""
    from cesm_emulator_amd.model import UNet, Diffusion
    torch.manual_seed(3)
    net = UNet(ch_mults=(1, 2, 4, 8)).to(dev)
    net.compute_dtype = torch.bfloat16
    d = Diffusion(net).to(dev)
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(2, 1, 64, 96, generator=g).to(dev)
    cond = torch.randn(2, 1, 12, 64, 96, generator=g).to(dev)
    t = torch.randint(0, 1000, (2,), generator=g).to(dev)
    noise = torch.randn(2, 1, 64, 96, generator=g).to(dev)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    loss = d.loss(x0, cond, t=t, noise=noise)
    loss.backward()
    torch.cuda.synchronize()
    out = {"variant": "train_step", "loss": loss.detach().cpu(),
           "peak_bytes": torch.tensor(torch.cuda.max_memory_allocated(dev) - base)}
    out.update({"grad." + n: p.grad.detach().cpu() for n, p in net.named_parameters() if p.grad is not None})
    return out


def compute(case, dev):
    if case == "train_step":
        return train_step_case(dev)
    return conv_case(case, dev) if case in CONV_CASES else tf_case(case, dev)


def main():
    case, path = sys.argv[1], sys.argv[2]
    dev = torch.device("cuda:0")
    torch.save(compute(case, dev), path)


if __name__ == "__main__":
    main()
