"""DDPM sampling throughput (inference.py:225-230 -> Diffusion.sample): one p_sample
step = F=1 forward of the full 192x288 grid + the fused update.  Times K steps of the eager loop
(model.py:186-194 semantics, one Python-driven launch sequence per step) and of the HIP-graph replay
(GraphSampleStep), and prints one JSON line.
usage: python tools/sample_bench.py [--config more_blocks] [--batch 8] [--steps 50] [--dtype bf16]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cesm_emulator_amd.model import Diffusion, GraphSampleStep  # noqa: E402
from cesm_emulator_amd.train import build_model_from_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="more_blocks")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--width", type=int, default=288)
    a = ap.parse_args()
    dev = torch.device("cuda")
    cfg = json.load(open(os.path.join(ROOT, "config", a.config)))
    torch.manual_seed(1)
    net = build_model_from_config(cfg["unet"]).to(dev)
    net.compute_dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    d = Diffusion(net).to(dev)
    B, H, W = a.batch, a.height, a.width
    cond = torch.randn(B, 1, H, W, device=dev)
    x = torch.randn(B, 1, H, W, device=dev)
    out = {"metric": "DDPM sampling steps/s (p_sample, F=1)", "config": a.config, "batch": B, "grid": [H, W],
           "dtype": a.dtype}
    with torch.inference_mode():
        # eager loop (reference control flow: host-side t tensor, randn_like, p_sample)
        for _ in range(3):
            x = d.p_sample(x, cond, torch.full((B,), 500, device=dev, dtype=torch.long))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            x = d.p_sample(x, cond, torch.full((B,), 999 - i, device=dev, dtype=torch.long))
        torch.cuda.synchronize()
        te = (time.perf_counter() - t0) / a.steps
        step = GraphSampleStep(d, cond, x)
        for _ in range(3):
            step.z.normal_()
            step.run(500)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step.z.normal_()
            step.run(999 - i)
        torch.cuda.synchronize()
        tg = (time.perf_counter() - t0) / a.steps
        assert torch.isfinite(step.x).all()
    out.update({"eager_ms_per_step": round(te * 1e3, 3), "graph_ms_per_step": round(tg * 1e3, 3),
                "graph_speedup": round(te / tg, 2), "graph_steps_per_s": round(1.0 / tg, 2),
                "fields_per_s_1000_steps": round(B / (1000 * tg), 4)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
