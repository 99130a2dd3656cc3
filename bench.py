#!/usr/bin/env python3
"""Benchmark: video_net training throughput on MI355X (BASELINE.json metric).

One step = one full training step of config/more_blocks on a per-GPU batch of synthetic
192x288 fields with F=12 frames: q_sample -> UNet fwd -> MSE -> bwd -> (RCCL grad all-reduce)
-> global-norm clip -> AdamW.  Inputs are resident in HBM before timing starts.

  python bench.py [--gpus N --steps K --warmup W --batch B --frames F --config more_blocks]
  N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Prints ONE JSON line (rank 0) with the contract fields plus `roofline` (dominant kernel, live HIP
events over the timed region) and `cpu_baseline` (oracle fp32 train step on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense BF16 MFMA (MI355X_MICROARCH.md, chip-level table)
PEAK_F32_TFLOPS = 157.3     # f32 MFMA
PEAK_HBM_GBS = 8000.0


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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-crop", type=int, default=4, help="cpu baseline runs on 1/crop of the grid")
    return ap.parse_args()


def load_cfg(name):
    with open(os.path.join(ROOT, "config", name)) as f:
        return json.load(f)


class KernelProbe:
    """Times every launch of the dominant kernel (level-0 3x3 conv forward, bf16 MFMA) with HIP
    events on the stream it is launched on, during the timed steps."""

    def __init__(self, kernels_mod, match):
        self.K = kernels_mod
        self.match = match
        self.events = []
        self.flops = []
        self.active = False
        self._orig = kernels_mod.conv_fwd

        def wrapped(x1, x2, wp, bias, geom, **kw):
            hit = self.active and self.match(x1, x2, geom)
            if hit:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
            y = self._orig(x1, x2, wp, bias, geom, **kw)
            if hit:
                e.record()
                Ho, Wo, Cout, KH, KW = geom[:5]
                cin = x1.shape[3] + (0 if x2 is None else x2.shape[3])
                self.events.append((s, e))
                self.flops.append(2.0 * x1.shape[0] * Ho * Wo * Cout * KH * KW * cin)
            return y

        kernels_mod.conv_fwd = wrapped

    def summary(self):
        if not self.events:
            return None
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e in self.events]
        avg_ms = sum(ms) / len(ms)
        avg_flops = sum(self.flops) / len(self.flops)
        return avg_ms, avg_flops, len(ms)


def pmc_traffic():
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes
    (tools/gpu_round.sh step 4 -> tools/traffic.py; FETCH_SIZE/WRITE_SIZE calibrated on a known copy)."""
    f = os.path.join(ROOT, "profiles", "r1_conv3x3_traffic.json")
    if not os.path.exists(f):
        return None, None
    with open(f) as fh:
        d = json.load(fh)
    return d["traffic_bytes_per_launch"], d["algorithmic_bytes_per_launch"]


def cpu_baseline(cfg_unet, F, H, W, crop):
    """Oracle fp32 train step (B=1) on the host cores, on a 1/crop spatial sample."""
    from oracle import ref_cpu as R
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    hh, ww = H // 2, W // 2  # 1/4 of the grid (96x144)
    if crop == 1:
        hh, ww = H, W
    torch.manual_seed(1)
    net = R.UNet(**R.config_unet_kwargs(cfg_unet))
    d = R.Diffusion(net)
    opt = R.make_optimizer(d)
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(1, 1, hh, ww, generator=g)
    cond = torch.randn(1, 1, F, hh, ww, generator=g)
    t0 = time.perf_counter()
    R.train_step(d, opt, x0, cond)
    dt = time.perf_counter() - t0
    scale = (H * W) / (hh * ww)
    return {"value": round(1.0 / (dt * scale), 6), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"1 oracle fp32 train step (fwd+bwd+clip+AdamW), B=1, F={F}, {hh}x{ww} spatial crop "
                      f"({dt:.1f}s), time scaled x{scale:.0f} to the {H}x{W} grid"}


def main():
    a = parse()
    from cesm_emulator_amd import distributed as D
    rank, local, world = D.setup()
    if world != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    import cesm_emulator_amd.kernels as K
    from cesm_emulator_amd.model import Diffusion
    from cesm_emulator_amd.optim import FusedAdamW
    from cesm_emulator_amd.train import build_model_from_config, train_step
    from cesm_emulator_amd.flops import train_flops_per_sample

    cfg = load_cfg(a.config)
    B, F, H, W = a.batch, a.frames, a.height, a.width
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    diff = Diffusion(unet).to(dev)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    dp = D.GradAllReducer() if world > 1 else None
    if dp is not None:
        dp.broadcast_params(opt.flat.data)

    # synthetic z-scored fields (train.py:640-646 semantics), resident in HBM, distinct per rank
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x0 = torch.randn(B, 1, H, W, device=dev, generator=g)
    cond = torch.randn(B, 1, F, H, W, device=dev, generator=g)

    # dominant kernel: the level-0 (full-grid, 64-ch) 3x3 conv forward
    probe = KernelProbe(K, lambda x1, x2, geom: geom[3] == 3 and x1.shape[1] == H and x1.shape[3] == 64
                        and x2 is None and geom[2] == 64)

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    t_w = time.perf_counter()
    for _ in range(a.warmup):
        train_step(diff, opt, x0, cond, 1.0, dp)
    torch.cuda.synchronize()
    log(f"warmup {a.warmup} steps: {time.perf_counter() - t_w:.1f}s, "
        f"peak mem {torch.cuda.max_memory_allocated(dev) / 2**30:.1f} GiB")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    probe.active = True
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = train_step(diff, opt, x0, cond, 1.0, dp)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    probe.active = False
    lval = float(loss.item())
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    samples = B * a.steps * world
    value = samples / elapsed
    tflop = train_flops_per_sample(unet.net, F, H, W) / 1e12
    peak = PEAK_BF16_TFLOPS if a.dtype == "bf16" else PEAK_F32_TFLOPS
    ps = probe.summary()
    roof = None
    if ps is not None:
        avg_ms, avg_flops, n = ps
        ach = avg_flops / (avg_ms * 1e-3) / 1e12
        traffic, alg_bytes = pmc_traffic() if a.dtype == "bf16" else (None, None)
        if traffic is not None:  # PMC passes run tools/conv_micro.py at B = 4; per-launch bytes scale with B
            traffic, alg_bytes = traffic * a.batch / 4, alg_bytes * a.batch / 4
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(ach / peak, 4), "traffic": traffic,
                "traffic_note": None if traffic is None else
                f"HBM bytes/launch (PMC FETCH_SIZE+WRITE_SIZE at B=4, profiles/r1_conv3x3_traffic.json, scaled "
                f"to B={a.batch}) vs {alg_bytes:.3g} algorithmic (input read + output write)",
                "kernel": "conv3x3p_kernel (level-0 3x3 conv 64->64, fwd+dgrad; persistent, resident weights)" if a.dtype == "bf16" else
                          "conv_fwd_kernel<float,64>", "launches": n, "avg_us": round(avg_ms * 1e3, 2),
                "flop_per_launch": avg_flops}
    out = {
        "metric": "train samples/sec (192x288xT frames)",
        "value": round(value, 4), "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.dtype, "data": "synthetic N(0,1) z-scored fields, resident in HBM",
        "config": {"workload": f"config/{a.config} train step, F={F}, {H}x{W}, per-GPU batch {B}",
                   "global_batch": B * world, "frames": F, "grid": [H, W], "parallelism": f"dp{world}"},
        "step_mfma": {"train_tflop_per_sample": round(tflop, 4),
                      "achieved_tflops": round(value * tflop, 2),
                      "frac_of_peak": round(value * tflop / peak, 4)},
        "loss": lval,
        "roofline": roof,
    }
    log(f"timed {a.steps} steps: {elapsed:.2f}s -> {value:.2f} samples/s")
    if not a.no_cpu_baseline and world == 1:
        log("cpu baseline (oracle fp32 train step on host cores) ...")
        out["cpu_baseline"] = cpu_baseline(cfg["unet"], F, H, W, a.cpu_crop)
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
