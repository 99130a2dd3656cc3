"""Diagnostic for the CESM_WGRAD_STREAM=1 slowdown: per-step wall time and the caching
allocator's counters (retries, device frees) of the bench step, with the knob as set in the environment.

  CESM_WGRAD_STREAM=1 python3 tools/wgrad_stream_diag.py [steps] [config] [B] [F]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from cesm_emulator_amd.model import Diffusion  # noqa: E402
from cesm_emulator_amd.optim import FusedAdamW  # noqa: E402
from cesm_emulator_amd.train import build_model_from_config, train_step  # noqa: E402
import json  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cname = sys.argv[2] if len(sys.argv) > 2 else "more_blocks"
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = json.load(open(os.path.join(ROOT, "config", cname)))
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    F = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    H, W = 192, 288
    g = torch.Generator(device=dev).manual_seed(1000)
    x0 = torch.randn(B, 1, H, W, device=dev, generator=g)
    cond = torch.randn(B, 1, F, H, W, device=dev, generator=g)
    keys = ["num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams",
            "allocated_bytes.all.peak", "reserved_bytes.all.current"]
    print(f"CESM_WGRAD_STREAM={os.environ.get('CESM_WGRAD_STREAM', '0')} {cname} B={B} F={F}", flush=True)
    for i in range(steps):
        s0 = torch.cuda.memory_stats(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        train_step(diff, opt, x0, cond, 1.0, None)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        s1 = torch.cuda.memory_stats(dev)
        d = {k: s1.get(k, 0) - s0.get(k, 0) for k in keys[:4]}
        print(f"step {i}: host enqueue {1e3 * (t1 - t0):.1f} ms, wall {1e3 * (t2 - t0):.1f} ms, "
              f"deltas {d}, peak {s1.get(keys[4], 0) / 2**30:.1f} GiB, reserved {s1.get(keys[5], 0) / 2**30:.1f} GiB",
              flush=True)


if __name__ == "__main__":
    main()
