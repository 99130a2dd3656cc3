"""Opt-in kernel variants behind environment knobs (INTEGRATION.md lists them as user knobs), each run in a child
process started with the knob set (the library reads a knob once per process) and compared with this process's
default kernels on the same seeded inputs (tests/knob_child.py computes both sides).

* CESM_CONV_WS=1 routes every bf16 3x3 conv whose 256-pixel tiles cover the image to >= 90 % through the
  warp-specialized conv3x3ws_kernel; by default only the level-0 64 -> 64 shape takes it (the rest measured slower).
  The opt-in shapes exercise its other paths: 128 / 256 channels (more than one 64-wide co block: weights streamed
  per step, the ws_decode co-block order, GroupNorm slots at cb * 16), concat inputs (x2 as the chunk source),
  Cout != Cin -- plain, with the fused residual, and with the GroupNorm-partial epilogue.
(Round 6 removed the other dispatch knobs and the code paths behind them: every alternative measured slower or
neutral -- DESIGN.md §6e lists them with their A/B records.  The remaining opt-in switches are CESM_CONV_WS (here),
CESM_CONV_STATIC (tests/test_gpu_prod_parity.py::test_conv3x3ws_dynamic_claim_bit_exact), CESM_WGRAD_STREAM (here)
and CESM_SAMPLE_GRAPH (tests/test_gpu_sampler.py).)
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


@pytest.mark.parametrize("mode", ["1", "attn"])
def test_wgrad_stream_opt_in_step(dev, tmp_path, mode):
    """CESM_WGRAD_STREAM=1 / attn: the weight gradients on a second HIP stream give the default step's loss and every
    gradient bit for bit (the same kernels on the same inputs, ordered after their producers), and the tensors the side
    stream reads are released level by level (RunCtx.checkpoint): at most the previous and the current
    level's tensors stay alive past their last use, so the step's peak memory stays within 25 % of the default's (measured
    1856 vs 1644 MiB with "1" at this shape; the whole-backward keep list of round 5 held every level's dy / x until
    the end)"""
    side = run_child("train_step", {"CESM_WGRAD_STREAM": mode}, tmp_path)
    ref = run_child("train_step", {"CESM_WGRAD_STREAM": "0"}, tmp_path)
    assert torch.equal(side["loss"], ref["loss"])
    names = [k for k in ref if k.startswith("grad.")]
    assert len(names) > 100 and sorted(names) == sorted(k for k in side if k.startswith("grad."))
    for k in names:
        assert torch.equal(side[k], ref[k]), k
    ps, pr = side["peak_bytes"].item(), ref["peak_bytes"].item()
    print(f"CESM_WGRAD_STREAM={mode}: peak {ps / 2**20:.0f} MiB vs default {pr / 2**20:.0f} MiB")
    assert ps <= 1.25 * pr, (ps, pr)
