#!/usr/bin/env python3
"""Benchmark: video_net training throughput on MI355X (BASELINE.json metric).

One step = one full training step of config/more_blocks on a per-GPU batch of synthetic
192x288 fields with F=12 frames: q_sample -> UNet fwd -> MSE -> bwd -> (RCCL grad all-reduce)
-> global-norm clip -> AdamW.  With the default --data resident the inputs are in HBM before timing
starts; --data device|pinned puts the training data path (dataset_single_member.py windows via the
HBM gather kernel, or host gather + pinned side-stream H2D) inside the timed region.

  python bench.py [--gpus N --steps K --warmup W --batch B --frames F --config more_blocks]
  N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Prints ONE JSON line (rank 0) with the contract fields plus
  roofline      the DOMINANT kernel by time per step: chosen from HIP events around every launch of the
                profiled ops in the last two warm-up steps, then timed live over the timed steps (events on the
                stream it runs on, around its launches only, so the timed region stays uninstrumented otherwise):
                algorithmic FLOP and bytes per launch, bound = the larger of the two floors, achieved / peak,
                PMC traffic measured at the bench batch (profiles/step_traffic.json);
  top_kernels   the five most expensive kernels by time per step (from the profiled warm-up steps), same fields;
  cpu_baseline  oracle fp32 train steps on the host cores;
  fwd_error     forward error of the HIP path vs the CPU oracle (the metric's "fwd MSE vs ref").
The last two come from the CPU leg (`cpu_leg`), the only part of this file that touches oracle/.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense BF16 MFMA (MI355X_MICROARCH.md, chip-level table)
PEAK_F32_TFLOPS = 157.3     # f32 MFMA
PEAK_HBM_GBS = 8000.0
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "step_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="samples per GPU per step (8 x 8 GPUs = config/more_blocks batch_size 64)")
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--width", type=int, default=288)
    ap.add_argument("--config", default="more_blocks", choices=["more_blocks", "baseline"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--data", default="resident", choices=["resident", "device", "pinned"],
                    help="resident: one synthetic batch in HBM; device/pinned: the training data path in the loop")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the CPU leg (cpu_baseline, fwd_error)")
    ap.add_argument("--cpu-full-configs", default="baseline,more_blocks",
                    help="comma list of configs whose full-grid oracle step is timed (D5), '' for none")
    ap.add_argument("--no-probe", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--dist-backend", default=None, choices=[None, "nccl", "gloo"],
                    help="torch.distributed backend for N>1 (default nccl = RCCL; gloo rehearses the multi-rank path "
                         "with several ranks on one GPU)")
    ap.add_argument("--other-configs", default="baseline_f12_b8,more_blocks_f120_b1,more_blocks_f12_b5",
                    help="extra single-GPU legs after the headline, outside its timed region (BASELINE.json configs "
                         "2, 4 and 5 per GPU; N=1 only); '' for none")
    return ap.parse_args()


# extra legs: name -> (config, per-GPU batch, frames, warm-up steps, timed steps, BASELINE.json config it stands for)
OTHER_CONFIGS = {
    "baseline_f12_b8": ("baseline", 8, 12, 3, 10, "configs[1]: config/baseline, 192x288x12, bf16, 1 GPU"),
    "more_blocks_f120_b1": ("more_blocks", 1, 120, 3, 5,
                            "configs[3] per-GPU leg: config/more_blocks, 192x288x120, 1 sample per GPU (8 GPUs DDP)"),
    "more_blocks_f12_b5": ("more_blocks", 5, 12, 3, 10,
                           "configs[4] per-GPU leg: config/more_blocks, 40-member batch over 8 GPUs = 5 per GPU"),
}


def load_cfg(name):
    with open(os.path.join(ROOT, "config", name)) as f:
        return json.load(f)


# ------------------------------------------------------------------------------------------------ probe
def _conv_work(K, x1, x2, geom, out_split):
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    Nb, Hi, Wi, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    cin = C1 + C2
    taps = KH * KW // (U * U)  # the transposed (U = 2) gather: a quarter of the taps are live per pixel
    es = x1.element_size()
    flop = 2.0 * Nb * Ho * Wo * Cout * taps * cin
    byt = float(es * (Nb * Hi * Wi * cin + Nb * Ho * Wo * Cout) + es * Cout * KH * KW * cin)
    return flop, byt


class KernelProbe:
    """HIP events around every launch of the profiled kernel wrappers (they enqueue on torch's current
    stream, which is where the events are recorded), with the algorithmic FLOP / bytes of each launch.
    Each wrapper is labelled with the kernel it launches (conv launches through the library's own
    dispatch query cesm_conv_*_variant); multi-kernel ops name their kernels."""

    def __init__(self, K):
        self.K = K
        self.active = False
        self.only = None  # set of labels to time (None: every profiled op)
        self.rec = []  # (label, start event, end event, flop, bytes)
        self._label_cache = {}
        self._orig = {}
        es_of = lambda t: t.element_size()  # noqa: E731

        def conv_fwd(x1, x2, wp, bias, geom, res=None, res2=None, out_split=None):
            Ho, Wo, Cout, KH, KW, St, Pd, U = geom
            Nb, Hi, Wi, C1 = x1.shape
            C2 = 0 if x2 is None else x2.shape[3]
            Co1 = Cout if out_split is None else out_split
            key = ("f", x1.dtype, Nb, Hi, Wi, C1, C2, Co1) + tuple(geom)
            lab = self._label_cache.get(key)
            if lab is None:
                lab = self._label_cache[key] = K.conv_fwd_variant(x1.dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1,
                                                                  KH, KW, St, Pd, U)
            f, b = _conv_work(K, x1, x2, geom, out_split)
            if res is not None:
                b += res.numel() * es_of(res) + (0 if res2 is None else res2.numel() * es_of(res2))
            return lab, f, b

        def conv_fwd_gn(x1, x2, wp, bias, geom, B, nslot):
            lab, f, b = conv_fwd(x1, x2, wp, bias, geom)
            return lab, f, b + B * nslot * geom[2] * 2  # + the GroupNorm partials (float2 per channel quad)

        def conv_wgrad(x1, x2, dy1, dy2, dw, geom, swap, flip, accumulate=True, db=None):
            Ho, Wo, Cout, KH, KW, St, Pd, U = geom
            Nb, Hi, Wi, C1 = x1.shape
            C2 = 0 if x2 is None else x2.shape[3]
            key = ("w", x1.dtype, Nb, Hi, Wi, C1, C2, dy1.shape[3], db is not None) + tuple(geom)
            lab = self._label_cache.get(key)
            if lab is None:
                lab = self._label_cache[key] = K.conv_wgrad_variant(
                    x1.dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, dy1.shape[3], KH, KW, St, Pd, U,
                    db is not None) + " + conv_wgrad_reduce_kernel"
            f, b = _conv_work(K, x1, x2, geom, None)  # same MACs as the forward; x and dY read, dW tiny
            return lab, f, b + dw.numel() * 4

        def tw_core_flop(C, F):  # per voxel: to_qkv + to_out GEMMs + q.k and attn.v
            return 2.0 * 768 * C + 2.0 * 256 * C + 2.0 * 2 * F * 32 * 8

        def tblock_fwd(x, gamma, wqkv, wout, bias, rot, B, F, scale, save=True, eps=1e-5, save_o=False):
            Nb, H, W, C = x.shape
            v = Nb * H * W
            nv = ({64: 4, 128: 2}.get(C, 1) * F + 15) // 16
            lab = f"tw_fwd_kernel<{C},{nv}>" if C <= 256 else f"tblock_fwd_kernel<{C}>"
            b = v * (2 * C * 2 + (40 if save else 0) + (512 if save_o else 0))
            return lab, v * tw_core_flop(C, F), float(b)

        def tblock_bwd(x, dy, gamma, mr, lse, wqkv, wqkv_t, wout_t, bias, rot, dgamma, dtable, B, F, scale,
                       want_wgrad_inputs=True, num_buckets=32, max_distance=32, emit_o=True):
            Nb, H, W, C = x.shape
            v = Nb * H * W
            nv = ({64: 4, 128: 2}.get(C, 1) * F + 15) // 16
            lab = (f"tw_bwd_kernel<{C},{nv}>" if C <= 256 else f"tblock_bwd_kernel<{C}>") + " (+ dgamma/dbias sums)"
            # dgrad-equivalent work (= the forward's FLOPs); bytes: x, dy read, mr/lse read, dx written, and the
            # weight-gradient inputs dqkv (768 ch), xn (and o when emitted) written
            b = v * (3 * C * 2 + 40)
            if want_wgrad_inputs:
                b += v * (768 * 2 + C * 2 + (512 if emit_o else 0))
            return lab, v * tw_core_flop(C, F), float(b)

        def tblock_fwd_fold(x, gamma, wqkv_f32, wout, bias, rot, B, F, scale, save=True, eps=1e-5, save_o=False):
            Nb, H, W, C = x.shape
            v = Nb * H * W
            nv = (4 * F + 15) // 16
            b = v * (2 * C * 2 + (40 if save else 0) + (512 if save_o else 0))
            return f"tw_fwd_kernel<{C},{nv},true>", v * tw_core_flop(C, F), float(b)

        def tblock_bwd_dw(x, dy, mr, lse, wqkv_f32, gamma, wout_t, bias, rot, dwqkv, dgamma, dtable, B, F, scale,
                          num_buckets=32, max_distance=32, emit_o=False):
            Nb, H, W, C = x.shape
            v = Nb * H * W
            nv = (4 * F + 15) // 16
            # dgrad-equivalent work (the forward's FLOPs) + the in-kernel to_qkv weight gradient (2 * 768 * C per
            # voxel; the O = P V recompute of emit_o is not counted); bytes: x, dy, mr / lse read, dx (and O) written
            return (f"twh_bwd_kernel<{nv}> (+ dW / dgamma / dbias reductions)",
                    v * (tw_core_flop(C, F) + 2.0 * 768 * C),
                    float(v * (3 * C * 2 + 40 + (512 if emit_o else 0))))

        def tattn_fwd(qkv, bias, rot, B, F, HW, scale, save=True, pixel_major=False):
            v = B * F * HW
            lab = (f"tflash_fwd2_kernel<{(F + 15) // 16}>" if K._tflash(qkv, F) else "tattn_fwd_kernel")
            # q.k and attn.v over the F frames of each pixel and head; bytes: qkv read, out (+ lse) written
            return lab, 4.0 * F * 32 * 8 * v, float(v * (768 * 2 + 256 * 2 + (32 if save else 0)))

        def tattn_bwd(qkv, o, dout, lse, bias, rot, dtable, B, F, HW, scale, num_buckets=32, max_distance=32,
                      pixel_major=False):
            v = B * F * HW
            nt = (F + 15) // 16
            # the kernel(s) by dispatch (cesm_tflash_bwd_variant): the one-pass fused backward (round 5), or the dq kernel
            # + the dk / dv kernel
            dq = K.tflash_bwd_variant(F, HW)  # the same selection for pixel-major qkv
            if not K._tflash(qkv, F):
                lab = "tattn_bwd_kernel"
            elif dq.startswith("tflash_bwd_fused"):
                lab = dq
            else:
                lab = f"{dq.replace(',false>', '>').replace(',true>', '>')} + tflash_bwd_kv_kernel<{nt}>"
            # dP, dQ, dK, dV products (2x the forward); bytes: qkv, o, dout, lse read once, dqkv written
            return lab, 8.0 * F * 32 * 8 * v, float(v * (768 * 2 * 2 + 256 * 2 * 2 + 32))

        def sla_flop(C):  # per voxel: to_qkv + to_out + context k v^T and context^T q (8 heads, 32 x 32)
            return 2.0 * 768 * C + 2.0 * 256 * C + 2.0 * 2 * 32 * 32 * 8

        def slaf_fwd(x, gamma, wqkv, wout, bout, scale, eps=1e-5, save_o=False):
            Nf, H, W, C = x.shape
            v = Nf * H * W
            return (f"slaf_stats_kernel<{C}> + slaf_combine_kernel + slaf_out_kernel<{C},{4 if C == 64 else 2}>",
                    v * sla_flop(C),
                    float(v * (2 * C * 2 + (512 if save_o else 0))))

        def slaf_bwd(x, dy, gamma, wqkv, wqkv_t, wout_t, state, dgamma, scale, want_wgrad_inputs=True, eps=1e-5):
            Nf, H, W, C = x.shape
            v = Nf * H * W
            b = v * 3 * C * 2 + (v * (768 * 2 + C * 2) if want_wgrad_inputs else 0)
            return (f"slab_dctx_kernel<{C}> + slab_combine_kernel + slab_dx_kernel<{C},{2 if C == 64 else 1}>",
                    v * sla_flop(C), float(b))

        def gn_stats(y, B, G, eps=1e-5):
            return "gn_stats_kernel", 0.0, float(y.numel() * es_of(y))

        def gn_stats_part(part, rows_b, G, eps=1e-5):
            return "gn_part_finalize_kernel", 0.0, float(part.numel() * 4)

        def gn_apply(y, stats, gamma, beta, ss, res, B, G):
            return "gn_apply_kernel", 0.0, float(y.numel() * es_of(y) * (3 if res is not None else 2))

        def gn_bwd(dout, y, stats, gamma, beta, ss, dgamma, dbeta, B, G, want_dss, dbias=None):
            # reduce pass reads dout, y; apply pass reads dout, y and writes dy
            return "gn_bwd_reduce_kernel + gn_bwd_apply_kernel", 0.0, float(y.numel() * es_of(y) * 5)

        def ln_fwd(x, gamma, save=True, eps=1e-5, perm=None):
            return "ln_fwd_kernel", 0.0, float(x.numel() * es_of(x) * 2)

        def ln_bwd(dy, x, mr, gamma, dgamma, dres=None, perm=None):
            return "ln_bwd_kernel", 0.0, float(x.numel() * es_of(x) * (4 if dres is not None else 3))

        def adamw(p, g, m, v, info, lr, b1, b2, eps, wd, step_dev, use_clip):
            return "adamw_kernel", 10.0 * p.numel(), float(p.numel() * 28)

        def add(a, b):
            return "add_kernel", 0.0, float(a.numel() * es_of(a) * 3)

        for name, fn in dict(conv_fwd=conv_fwd, conv_fwd_gn=conv_fwd_gn, conv_wgrad=conv_wgrad, tblock_fwd=tblock_fwd, tblock_bwd=tblock_bwd,
                             tblock_fwd_fold=tblock_fwd_fold, tblock_bwd_dw=tblock_bwd_dw,
                             tattn_fwd=tattn_fwd, tattn_bwd=tattn_bwd,
                             slaf_fwd=slaf_fwd, slaf_bwd=slaf_bwd, gn_stats=gn_stats, gn_stats_part=gn_stats_part, gn_apply=gn_apply, gn_bwd=gn_bwd,
                             ln_fwd=ln_fwd, ln_bwd=ln_bwd, adamw=adamw, add=add).items():
            self._wrap(name, fn)

    def _wrap(self, name, work):
        orig = getattr(self.K, name)
        self._orig[name] = orig

        def wrapped(*a, **kw):
            if not self.active:
                return orig(*a, **kw)
            lab, f, b = work(*a, **kw)
            if self.only is not None and lab not in self.only:
                return orig(*a, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = orig(*a, **kw)
            e.record()
            self.rec.append((lab, s, e, f, b))
            return out

        setattr(self.K, name, wrapped)

    def reset(self):
        torch.cuda.synchronize()
        self.rec = []

    def table(self, steps, peak_tflops, traffic):
        torch.cuda.synchronize()
        agg = {}
        for lab, s, e, f, b in self.rec:
            a = agg.setdefault(lab, [0, 0.0, 0.0, 0.0])
            a[0] += 1
            a[1] += s.elapsed_time(e)
            a[2] += f
            a[3] += b
        rows = []
        for lab, (n, ms, f, b) in agg.items():
            sec = ms * 1e-3
            t_mfma, t_hbm = f / (peak_tflops * 1e12), b / (PEAK_HBM_GBS * 1e9)
            bound = "mfma" if t_mfma >= t_hbm else "hbm"
            ach_tf, ach_gb = f / sec / 1e12, b / sec / 1e9
            row = {"kernel": lab, "ms_per_step": round(ms / steps, 3), "launches_per_step": round(n / steps, 2),
                   "avg_us": round(ms / n * 1e3, 2), "flop_per_launch": f / n, "bytes_per_launch": b / n,
                   "tflops": round(ach_tf, 2), "gbs": round(ach_gb, 1), "bound": bound,
                   "frac": round(ach_tf / peak_tflops if bound == "mfma" else ach_gb / PEAK_HBM_GBS, 4)}
            row["traffic"] = _traffic_lookup(lab, traffic)
            rows.append(row)
        rows.sort(key=lambda r: -r["ms_per_step"])
        return rows


def _traffic_lookup(label, kernels):
    """PMC bytes per launch of an op = the sum over the kernels its label names (each: exact demangled name,
    else the same template with trailing default arguments, conv3x3p_kernel<32,7,true> ->
    conv3x3p_kernel<32,7,true,2,10>, or for a name without template arguments the same base name);
    None if any of them has no PMC entry"""
    if not kernels:
        return None
    total = 0.0
    for k in re.split(r" \+ ", re.split(r" \(", label)[0]):
        k = k.strip()
        if k in kernels:
            total += kernels[k]["bytes_per_launch"]
            continue
        base, _, args = k.partition("<")
        args = args.rstrip(">")
        c = [n for n in kernels if n.split("<")[0] == base and (not args or n.startswith(f"{base}<{args},"))]
        if not c:
            return None
        total += max((kernels[n] for n in c), key=lambda e: e["launches_per_step"])["bytes_per_launch"]
    return total


def load_traffic(batch, frames, config):
    """per-kernel HBM bytes per launch from the committed PMC passes over this bench's own step
    (tools/step_pmc.py + tools/step_traffic.py: FETCH_SIZE x2 and WRITE_SIZE, calibrated on a known copy),
    only if they were measured at this batch / window / config"""
    if not os.path.exists(TRAFFIC_FILE):
        return None
    with open(TRAFFIC_FILE) as fh:
        d = json.load(fh)
    if (d.get("batch"), d.get("frames"), d.get("config")) != (batch, frames, config):
        return None
    return d["kernels"]


# ------------------------------------------------------------------------------------------------ CPU leg
def _cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_leg(dev, full_configs):
    """The bench's only use of oracle/ (test infrastructure, the checker — never the thing measured on the GPU):
      cpu_baseline: the oracle's fp32 train step (fwd + bwd + clip + AdamW, train.py:868-880 semantics) on the host
        cores per SURVEY.md §8(d) D5 — config 1 (baseline, F=8, 32x48, B=2): 3 warm-up + 10 timed steps; then ONE
        timed full-grid step (192x288, F=12, B=1) of each config in `full_configs`; no extrapolation.
        value = the more_blocks full-grid step (the bench workload), in samples/s.
      fwd_error: UNet forward of the HIP path vs the oracle on config 1's shapes (fp32 kernel mode: the north-star
        gate < 1e-5; bf16 reported)."""
    from oracle import ref_cpu as R
    from cesm_emulator_amd.model import UNet
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)

    def make(cfg_name, B, F, H, W, seed=1):
        torch.manual_seed(seed)
        net = R.UNet(**R.config_unet_kwargs(load_cfg(cfg_name)["unet"]))
        d = R.Diffusion(net)
        opt = R.make_optimizer(d)
        g = torch.Generator().manual_seed(0)
        x0 = torch.randn(B, 1, H, W, generator=g)
        cond = torch.randn(B, 1, F, H, W, generator=g)
        return net, d, opt, x0, cond

    # --- forward error on config 1 shapes (baseline, F = 8, 32 x 48, B = 2)
    net, d, opt, x0, cond = make("baseline", 2, 8, 32, 48)
    t = torch.tensor([17, 801])
    xt = torch.randn_like(x0)
    prod = UNet(**R.config_unet_kwargs(load_cfg("baseline")["unet"]))
    prod.load_state_dict(net.state_dict())
    prod = prod.to(dev)
    with torch.no_grad():
        y_ref = net(xt, cond, t).double()
        errs = {}
        for dt in (torch.float32, torch.bfloat16):
            prod.compute_dtype = dt
            y = prod(xt.to(dev), cond.to(dev), t.to(dev)).double().cpu()
            errs[dt] = ((y - y_ref).norm() / y_ref.norm()).item(), ((y - y_ref) ** 2).mean().item()
    del prod
    fwd_error = {"config": "config/baseline (config 1 shapes: F=8, 32x48, B=2), same weights and inputs",
                 "fp32_rel_l2": errs[torch.float32][0], "fp32_mse": errs[torch.float32][1],
                 "bf16_rel_l2": errs[torch.bfloat16][0], "bf16_mse": errs[torch.bfloat16][1],
                 "gate": "fp32 rel_l2 < 1e-5 (BASELINE.json north_star)",
                 "pass": errs[torch.float32][0] < 1e-5}

    # --- config 1 train steps: 3 warm-up + 10 timed
    for _ in range(3):
        R.train_step(d, opt, x0, cond)
    t0 = time.perf_counter()
    n1 = 10
    for _ in range(n1):
        R.train_step(d, opt, x0, cond)
    c1 = time.perf_counter() - t0
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    # cores = the intra-op threads the oracle actually ran with; the machine's logical CPUs and this process's
    # affinity mask are recorded beside it (the GPU box caps OMP_NUM_THREADS at 16 on a many-core host)
    out = {"unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port", "cpu_model": _cpu_model_name(),
           "os_cpu_count": os.cpu_count(), "sched_affinity_cpus": affinity,
           "config1_samples_per_s": round(2 * n1 / c1, 4),
           "config1_sample": f"config/baseline F=8 32x48 B=2: 3 warm-up + {n1} timed steps, {c1:.2f}s"}
    full = {}
    for name in [c for c in full_configs.split(",") if c]:
        net, d, opt, x0, cond = make(name, 1, 12, 192, 288)
        t0 = time.perf_counter()
        R.train_step(d, opt, x0, cond)
        dt = time.perf_counter() - t0
        full[name] = (dt, 1.0 / dt)
        del net, d, opt
    if "more_blocks" in full:
        out["value"] = round(full["more_blocks"][1], 6)
        out["sample"] = (f"1 timed oracle fp32 train step (fwd+bwd+clip+AdamW) of config/more_blocks on the full "
                         f"192x288 grid, F=12, B=1 ({full['more_blocks'][0]:.1f}s), after the config-1 warm-up; "
                         f"not extrapolated")
    else:
        out["value"] = out["config1_samples_per_s"]
        out["sample"] = out["config1_sample"]
    for name, (dt, v) in full.items():
        out[f"full_grid_{name}_samples_per_s"] = round(v, 6)
    return out, fwd_error


# ------------------------------------------------------------------------------------------------ data feeds
def make_feed(kind, B, F, H, W, dev, rank, world, steps_total):
    """iterator of (cond [B,1,F,H,W], x0 [B,1,H,W]) for --data device|pinned: synthetic z-scored
    (T, M, H, W) fields (M = 40 CESM-LE members), windows drawn as dataset_single_member.py does"""
    import numpy as np
    from cesm_emulator_amd import data as DA
    M = 40
    need = steps_total * B * world
    T = F + max(1, -(-need // M))
    r = np.random.default_rng(100)
    cond = r.standard_normal((T, M, H, W), dtype=np.float32)
    tgt = r.standard_normal((T, M, H, W), dtype=np.float32)
    cls = DA.DeviceWindowLoader if kind == "device" else DA.PinnedWindowLoader
    ld = cls(cond, tgt, F, B, dev, time_reverse_p=0.5, seed=0, rank=rank, world=world)
    np.random.seed(rank)

    def gen():
        epoch = 0
        while True:
            ld.set_epoch(epoch)
            for c, x in ld:
                if c.shape[0] == B:
                    yield c, x
            epoch += 1
    return gen()


# ------------------------------------------------------------------------------------------------ timing
def roofline_obj(d, steps, elapsed, peak):
    """the contract's roofline object from a KernelProbe.table row of the dominant kernel"""
    return {"bound": d["bound"],
            "achieved": d["gbs"] if d["bound"] == "hbm" else d["tflops"],
            "peak": PEAK_HBM_GBS if d["bound"] == "hbm" else peak,
            "unit": "GB/s" if d["bound"] == "hbm" else "TFLOP/s",
            "frac": d["frac"], "traffic": d["traffic"],
            "kernel": d["kernel"], "launches": int(round(d["launches_per_step"] * steps)),
            "avg_us": d["avg_us"], "ms_per_step": d["ms_per_step"],
            "share_of_step": round(d["ms_per_step"] / (elapsed / steps * 1e3), 4),
            "flop_per_launch": d["flop_per_launch"], "bytes_per_launch": d["bytes_per_launch"],
            "traffic_note": ("PMC FETCH_SIZE (x2, gfx950) + WRITE_SIZE bytes per launch at this batch, copy-calibrated "
                             f"({os.path.relpath(TRAFFIC_FILE, ROOT)})") if d["traffic"] is not None else
                            "no PMC pass at this batch/config"}


def other_leg(name, dev, probe, log):
    """One extra single-GPU leg (OTHER_CONFIGS): resident synthetic batch, W warm-up steps (the last two profile
    every kernel, choosing the dominant one), K timed steps bracketed by synchronize, the dominant kernel timed
    live (as the headline).  Returns samples/s, ms/step, the step's MFMA fraction and the dominant-kernel roofline."""
    from cesm_emulator_amd.model import Diffusion
    from cesm_emulator_amd.optim import FusedAdamW
    from cesm_emulator_amd.train import build_model_from_config, train_step, rank_generator
    from cesm_emulator_amd.flops import train_flops_per_sample
    cfg_name, B, F, warm, steps, what = OTHER_CONFIGS[name]
    H, W = 192, 288
    torch.manual_seed(1)
    unet = build_model_from_config(load_cfg(cfg_name)["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    diff.generator = rank_generator(dev, 2, 0)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(1000)
    x0 = torch.randn(B, 1, H, W, device=dev, generator=g)
    cond = torch.randn(B, 1, F, H, W, device=dev, generator=g)
    torch.cuda.reset_peak_memory_stats(dev)
    top_rows = None
    if probe is not None:
        probe.only = None
    for i in range(warm):
        if probe is not None and i == warm - 2:
            probe.reset()
            probe.active = True
        train_step(diff, opt, x0, cond, 1.0, None)
    torch.cuda.synchronize()
    if probe is not None:
        probe.active = False
        top_rows = probe.table(2, PEAK_BF16_TFLOPS, load_traffic(B, F, cfg_name))
        probe.only = {top_rows[0]["kernel"]}
        probe.reset()
        probe.active = True
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = train_step(diff, opt, x0, cond, 1.0, None)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    res = {"config": f"config/{cfg_name}, F={F}, {H}x{W}, per-GPU batch {B}", "stands_for": what,
           "steps": steps, "warmup": warm, "samples_per_s": round(B * steps / elapsed, 4),
           "ms_per_step": round(elapsed / steps * 1e3, 3), "loss": float(loss.item()),
           "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)}
    tflop = train_flops_per_sample(unet.net, F, H, W) / 1e12
    res["step_mfma"] = {"train_tflop_per_sample": round(tflop, 4), "achieved_tflops": round(B * steps / elapsed * tflop, 2),
                        "frac_of_peak": round(B * steps / elapsed * tflop / PEAK_BF16_TFLOPS, 4)}
    if probe is not None:
        probe.active = False
        rows = probe.table(steps, PEAK_BF16_TFLOPS, load_traffic(B, F, cfg_name))
        res["roofline"] = roofline_obj(rows[0], steps, elapsed, PEAK_BF16_TFLOPS)
        res["top_kernels"] = [{k: r[k] for k in ("kernel", "ms_per_step", "avg_us", "tflops", "gbs", "frac")}
                              for r in top_rows[:5]]
        probe.reset()
        probe.only = None
    log(f"{name}: {res['samples_per_s']:.3f} samples/s ({res['ms_per_step']:.1f} ms/step), "
        f"step MFMA {res['step_mfma']['frac_of_peak']:.3f}")
    del diff, opt, unet, x0, cond
    torch.cuda.empty_cache()
    return res


# ------------------------------------------------------------------------------------------------ main
def main():
    a = parse()
    from cesm_emulator_amd import distributed as D
    rank, local, world = D.setup(backend=a.dist_backend)
    if world != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    ndev = torch.cuda.device_count()
    if local >= ndev:  # more ranks than GPUs (a gloo rehearsal): ranks share the devices round-robin
        print(f"[bench] rank {rank}: LOCAL_RANK {local} >= {ndev} devices, using cuda:{local % ndev}", file=sys.stderr)
        local = local % ndev
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    import cesm_emulator_amd.kernels as K
    from cesm_emulator_amd.model import Diffusion
    from cesm_emulator_amd.optim import FusedAdamW
    from cesm_emulator_amd.train import build_model_from_config, train_step, rank_generator
    from cesm_emulator_amd.flops import train_flops_per_sample

    cfg = load_cfg(a.config)
    B, F, H, W = a.batch, a.frames, a.height, a.width
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    diff = Diffusion(unet).to(dev)
    diff.generator = rank_generator(dev, 2, rank)  # t / eps stream per rank
    opt = FusedAdamW(diff.parameters(), lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    dp = D.GradAllReducer() if world > 1 else None
    if dp is not None:
        dp.broadcast_params(opt.flat.data)

    if a.data == "resident":
        # synthetic z-scored fields (train.py:640-646 semantics), resident in HBM, distinct per rank
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        x0 = torch.randn(B, 1, H, W, device=dev, generator=g)
        cond = torch.randn(B, 1, F, H, W, device=dev, generator=g)
        next_batch = lambda: (cond, x0)  # noqa: E731
    else:
        feed = make_feed(a.data, B, F, H, W, dev, rank, world, a.warmup + a.steps)
        next_batch = lambda: next(feed)  # noqa: E731

    probe = None if a.no_probe else KernelProbe(K)

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    # Kernel profile in two parts, so the timed region carries almost no instrumentation: the last (up to 2)
    # warm-up steps time EVERY profiled op (-> top_kernels and the choice of the dominant kernel); the timed
    # steps then time only the dominant kernel's launches (-> roofline, live over the timed region).
    n_prof = min(2, max(0, a.warmup - 1)) if probe is not None else 0
    t_w = time.perf_counter()
    for i in range(a.warmup):
        if probe is not None and i == a.warmup - n_prof:
            probe.reset()
            probe.active = True
        c, x = next_batch()
        train_step(diff, opt, x, c, 1.0, dp)
    torch.cuda.synchronize()
    top_rows = None
    if probe is not None:
        probe.active = False
        if n_prof > 0:
            peak0 = PEAK_BF16_TFLOPS if a.dtype == "bf16" else PEAK_F32_TFLOPS
            top_rows = probe.table(n_prof, peak0, load_traffic(B, F, a.config) if a.dtype == "bf16" else None)
            probe.only = {top_rows[0]["kernel"]}
        probe.reset()
    log(f"warmup {a.warmup} steps: {time.perf_counter() - t_w:.1f}s, "
        f"peak mem {torch.cuda.max_memory_allocated(dev) / 2**30:.1f} GiB")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    if probe is not None:
        probe.active = True
    if dp is not None:
        dp.pop_timing()
        dp.timing = True  # HIP events around each bucket on the communication stream (no host sync in the loop)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        c, x = next_batch()
        loss = train_step(diff, opt, x, c, 1.0, dp)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if probe is not None:
        probe.active = False
    lval = float(loss.item())
    dist_info = None
    if world > 1:
        ar_ms, ar_n, ar_bytes = dp.pop_timing()
        dp.timing = False
        # what the ranks saw: world size, backend, RCCL version, and the all-reduce time per step (max over ranks,
        # from the events on the communication stream -- overlapped with the backward, so not additive to the step)
        tt = torch.tensor([elapsed, ar_ms / a.steps], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed, ar_ms_step = float(tt[0].item()), float(tt[1].item())
        try:
            ver = torch.cuda.nccl.version()
            ver = ".".join(map(str, ver)) if isinstance(ver, tuple) else str(ver)
        except Exception as e:  # noqa: BLE001 - reported, not fatal
            ver = f"unavailable ({type(e).__name__})"
        dist_info = {"world_size": torch.distributed.get_world_size(), "backend": torch.distributed.get_backend(),
                     "rccl_version": ver, "allreduce_ms_per_step": round(ar_ms_step, 3),
                     "allreduce_buckets_per_step": ar_n // a.steps, "allreduce_mb_per_step": round(ar_bytes / a.steps / 2**20, 1),
                     "bucket_mb": dp.bucket_elems * 4 / 2**20}

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    samples = B * a.steps * world
    value = samples / elapsed
    tflop = train_flops_per_sample(unet.net, F, H, W) / 1e12
    peak = PEAK_BF16_TFLOPS if a.dtype == "bf16" else PEAK_F32_TFLOPS
    roof, top = None, None
    if probe is not None:
        rows = probe.table(a.steps, peak, load_traffic(B, F, a.config) if a.dtype == "bf16" else None)
        top = (top_rows or rows)[:5]
        roof = roofline_obj(rows[0], a.steps, elapsed, peak)
    out = {
        "metric": "train samples/sec (192x288xT frames)",
        "value": round(value, 4), "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.dtype,
        "data": ("synthetic N(0,1) z-scored fields, resident in HBM" if a.data == "resident" else
                 f"synthetic (T, 40 members, H, W) fields through the {a.data} window loader inside the timed region"),
        "config": {"workload": f"config/{a.config} train step, F={F}, {H}x{W}, per-GPU batch {B}",
                   "global_batch": B * world, "frames": F, "grid": [H, W], "parallelism": f"dp{world}"},
        "step_mfma": {"train_tflop_per_sample": round(tflop, 4),
                      "achieved_tflops": round(value * tflop, 2),
                      "frac_of_peak": round(value * tflop / peak, 4)},
        "loss": lval,
        "roofline": roof,
        "top_kernels": top,
    }
    if dist_info is not None:
        out["distributed"] = dist_info
    log(f"timed {a.steps} steps: {elapsed:.2f}s -> {value:.2f} samples/s")
    if world == 1 and a.other_configs and a.dtype == "bf16":
        # BASELINE.json configs 2, 4 (per-GPU leg) and 5 (per-GPU batch), after the headline and outside its timed
        # region; the headline's model, optimizer state and batch are freed first
        del diff, opt, unet, next_batch
        if a.data == "resident":
            del cond, x0
        torch.cuda.empty_cache()
        out["other_configs"] = {}
        for name in [n for n in a.other_configs.split(",") if n]:
            out["other_configs"][name] = other_leg(name, dev, probe, log)
    if not a.no_cpu_baseline and world == 1:
        log("CPU leg (oracle fp32: forward error, train steps on host cores) ...")
        out["cpu_baseline"], out["fwd_error"] = cpu_leg(dev, a.cpu_full_configs)
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
