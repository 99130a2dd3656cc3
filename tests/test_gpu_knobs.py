"""Opt-in kernel variants behind environment knobs (INTEGRATION.md lists them as user knobs), each run in a child
process started with the knob set (the library reads a knob once per process) and compared with this process's
default kernels on the same seeded inputs (tests/knob_child.py computes both sides).

* CESM_CONV_WS=1 routes every bf16 3x3 conv whose 256-pixel tiles cover the image to >= 90 % through the
  warp-specialized conv3x3ws_kernel; by default only the level-0 64 -> 64 shape takes it (the rest measured slower).
  The opt-in shapes exercise its other paths: 128 / 256 channels (more than one 64-wide co block: weights streamed
  per step, the ws_decode co-block order, GroupNorm slots at cb * 16), concat inputs (x2 as the chunk source),
  Cout != Cin -- plain, with the fused residual, and with the GroupNorm-partial epilogue.
* CESM_TF_QW=1 selects the per-wave dq kernel (tflash_bwd_qw_kernel) of the long-window attention backward, for
  frame-major and pixel-major qkv rows (the latter is the F > 16 path's default layout).
"""
import os
import subprocess
import sys

import pytest
import torch

from tests import knob_child as KC

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel(a, b):
    a, b = a.double(), b.double()
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b).clamp_min(1e-30)).item()


def run_child(case, env, tmp_path):
    out = tmp_path / f"{case}.pt"
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "knob_child.py"), case, str(out)], cwd=ROOT,
                       env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("case", sorted(KC.CONV_CASES))
def test_conv_ws_opt_in_shapes(dev, tmp_path, case):
    """CESM_CONV_WS=1: conv3x3ws against the halo conv the default dispatch picks.  Both sum the same bf16
    products in fp32 in an order that gives the same bits (measured: y bit-exact), but the warp-specialized
    epilogue adds the fused residual to the bf16-ROUNDED conv output it staged in LDS (two roundings), the halo conv
    to the fp32 sum (one): y + res may differ by one bf16 rounding of y plus one of the sum -- relative to a sum that
    cancels, many of its ulps (measured rel 2.5e-3 at c128).  Gates: |a - b| <= 2^-8 (|y| + |a| + |b|) per element
    (+ fp32 summation noise), rel 4e-3 for y + res; y and the GroupNorm launch's y within one ulp (rel 2e-3); the
    conv_fwd_gn launch must store the same y as the plain launch, and its GroupNorm partials must give the separate
    statistics pass's (mean, rstd) to summation order"""
    ws = run_child(case, {"CESM_CONV_WS": "1"}, tmp_path)
    ref = KC.compute(case, dev)
    assert ws["variant"].startswith("conv3x3ws_kernel"), ws["variant"]
    assert not ref["variant"].startswith("conv3x3ws_kernel"), ref["variant"]
    for k in ("y", "y_res", "y_gn"):
        a, b = ws[k].float(), ref[k].float()
        noise = 1e-4 * b.pow(2).mean().sqrt()  # fp32 summation noise for outputs that cancel to near zero
        if k == "y_res":
            bound = (ref["y"].float().abs() + a.abs() + b.abs()) * 2.0 ** -8 + noise
        else:
            bound = torch.maximum(a.abs(), b.abs()) * 2.0 ** -7 + noise  # one bf16 ulp of the larger value
        worst = ((a - b).abs() / bound).max().item()
        e = rel(a, b)
        print(f"{case} {k}: {ws['variant']} vs {ref['variant']}: rel {e:.2e}, worst {worst:.2f} of the bound, "
              f"bit-exact {torch.equal(ws[k], ref[k])}")
        assert e < (4e-3 if k == "y_res" else 2e-3) and worst <= 1.0, (k, e, worst)
    assert torch.equal(ws["y_gn"], ws["y"])
    for side in (ws, ref):
        st, st0 = side["gn_stats"].double(), side["gn_stats_ref"].double()
        dm = ((st[..., 0] - st0[..., 0]).abs() * st0[..., 1]).max().item()
        dr = ((st[..., 1] - st0[..., 1]).abs() / st0[..., 1]).max().item()
        assert dm < 1e-5 and dr < 1e-5, (side["variant"], dm, dr)


@pytest.mark.parametrize("case", sorted(c for c, (F, _, _) in KC.TF_CASES.items() if F > 16))
def test_tflash_qw_opt_in(dev, tmp_path, case):
    """CESM_TF_QW=1: the per-wave dq kernel against the default block kernels, frame-major and pixel-major qkv rows
    (dq from sum P dP per wave vs D = dO . O: different summation, hence a tolerance; dk / dv and the bias-table
    gradient come from the same kv kernel but its dS input differs by dq's rounding path)"""
    qw = run_child(case, {"CESM_TF_QW": "1"}, tmp_path)
    ref = KC.compute(case, dev)
    F, HW, _ = KC.TF_CASES[case]
    assert qw["variant"].startswith("tflash_bwd_qw_kernel"), qw["variant"]
    assert not ref["variant"].startswith("tflash_bwd_qw_kernel"), ref["variant"]
    for k, kt in (("dqkv", "dtable"), ("dqkv_pm", "dtable_pm")):
        e, et = rel(qw[k].float(), ref[k].float()), rel(qw[kt], ref[kt])
        eq = rel(qw[k][:, :256].float(), ref[k][:, :256].float())
        print(f"{case} F={F} HW={HW} {k}: rel dqkv {e:.2e} (dq {eq:.2e}) dtable {et:.2e}")
        assert e < 1e-2 and et < 1e-3, (k, e, et)
        assert torch.isfinite(qw[k].float()).all()


@pytest.mark.parametrize("case", sorted(KC.TF_CASES))
def test_tflash_two_kernel_opt_in(dev, tmp_path, case):
    """CESM_TF_FUSED=0: the round-2..4 two-kernel long-window backward (dq kernel + dk / dv kernel) against the default
    one-pass fused kernel (round 5), frame-major and pixel-major qkv rows.  Both take D = dO . O at F > 16; the fused
    kernel rounds P and dS to bf16 once per tile where the two kernels do it per kernel, hence a tolerance.  At F <= 16
    the two-kernel form takes D = sum P dP (exact) against the fused kernel's D = dO . O from the bf16 O: the bias-table
    gradient, a sum of dS, differs by up to ~2e-3 there (both are checked against float64 in test_gpu_kernels.py)."""
    two = run_child(case, {"CESM_TF_FUSED": "0"}, tmp_path)
    ref = KC.compute(case, dev)
    F, HW, _ = KC.TF_CASES[case]
    assert ref["variant"].startswith("tflash_bwd_fused_kernel"), ref["variant"]
    assert not two["variant"].startswith("tflash_bwd_fused_kernel"), two["variant"]
    for k, kt in (("dqkv", "dtable"), ("dqkv_pm", "dtable_pm")):
        if k not in two:
            continue
        e, et = rel(two[k].float(), ref[k].float()), rel(two[kt], ref[kt])
        print(f"{case} F={F} HW={HW} {k}: {two['variant']} vs {ref['variant']}: rel dqkv {e:.2e} dtable {et:.2e}")
        assert e < 1e-2 and et < (1e-3 if F > 16 else 3e-3), (k, e, et)
        assert torch.isfinite(ref[k].float()).all()
