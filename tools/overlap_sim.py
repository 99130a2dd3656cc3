"""One-GPU measurement of the data-parallel step with its gradient all-reduce overlapped with the backward (VERDICT r4
item 5): the bench workload (config/more_blocks, F = 12, 192 x 288, B = 8 per GPU, bf16) timed as
  plain    -- train_step without data parallelism (the 1-GPU bench step);
  overlap  -- train_step with distributed.XgmiModelReducer: each 32-MB bucket's RCCL all-reduce replaced by
              cesm_hold_cus, `cus` blocks holding whole CUs on the communication stream for the bucket's modelled
              8-GPU ring time (busbw GB/s), issued during the backward exactly where the RCCL calls go;
  serial   -- the same holds on the compute stream after the backward (no overlap: the cost to hide);
each with the persistent level-0 conv's dynamic item claiming (default) and with its static split (CESM_CONV_STATIC),
alternating, `reps` times.  Prints one line per run and a JSON summary (ratios to the plain step).

  python tools/overlap_sim.py [--steps 10] [--warmup 3] [--cus 16,32] [--busbw 300] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--cus", default="16,32")
    ap.add_argument("--busbw", type=float, default=300.0)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import cesm_emulator_amd.kernels as K
    from cesm_emulator_amd.distributed import XgmiModelReducer
    from cesm_emulator_amd.model import Diffusion
    from cesm_emulator_amd.optim import FusedAdamW
    from cesm_emulator_amd.train import build_model_from_config, train_step, rank_generator
    dev = torch.device("cuda:0")
    with open(os.path.join(ROOT, "config", "more_blocks")) as f:
        cfg = json.load(f)
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    diff.generator = rank_generator(dev, 2, 0)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, max_grad_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(1000)
    B = a.batch
    x0 = torch.randn(B, 1, 192, 288, device=dev, generator=g)
    cond = torch.randn(B, 1, 12, 192, 288, device=dev, generator=g)
    nbytes = opt.flat.grad.numel() * 4

    def run(mode, cus, static):
        K.STATIC_CONV = static
        dp = None
        if mode != "plain":
            dp = XgmiModelReducer(world=8, cus=cus, busbw_gbs=a.busbw)
            dp.overlap = mode == "overlap"
        for _ in range(a.warmup):
            train_step(diff, opt, x0, cond, 1.0, dp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            train_step(diff, opt, x0, cond, 1.0, dp)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        held = sum(dp.issued_us) / (a.warmup + a.steps) / 1e3 if dp is not None else 0.0
        return ms, held

    cus_list = [int(c) for c in a.cus.split(",") if c]
    runs = [("plain", 0, False), ("plain", 0, True)]
    for c in cus_list:
        runs += [("overlap", c, False), ("overlap", c, True), ("serial", c, False)]
    res = {}
    for rep in range(a.reps):
        for mode, cus, static in runs:
            ms, held = run(mode, cus, static)
            key = f"{mode}{'' if mode == 'plain' else f'_cus{cus}'}_{'static' if static else 'dynamic'}"
            res.setdefault(key, []).append(ms)
            print(f"rep {rep} {key}: {ms:.2f} ms/step (modelled all-reduce {held:.2f} ms/step)", flush=True)
    best = {k: min(v) for k, v in res.items()}
    base = {"dynamic": best["plain_dynamic"], "static": best["plain_static"]}
    summary = {"workload": f"config/more_blocks train step, F=12, 192x288, B={B}, bf16",
               "grad_bytes": nbytes, "bucket_bytes": 32 << 20, "model": f"8-GPU ring, busbw {a.busbw} GB/s",
               "modelled_allreduce_ms_per_step": round(2 * 7 / 8 * nbytes / (a.busbw * 1e6), 3),
               "ms_per_step_best": {k: round(v, 2) for k, v in best.items()},
               "ratio_to_plain": {k: round(v / base[k.rsplit("_", 1)[1]], 4) for k, v in best.items()}}
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
