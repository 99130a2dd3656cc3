"""The CESM_WGRAD_STREAM=1 slowdown, reproduced as bench.py has it: legs in ONE process --
  leg A: more_blocks F = 12, B = 8 (the bench's main leg), then
  leg B: baseline F = 12, B = 8 (bench's first `other_configs` leg, after freeing leg A and empty_cache()),
each with warm-up + timed steps, the caching allocator's counters around the timed steps, and a marker kernel
(cesm_hold_cus, 1 block, 1 us) before each leg's timed steps so a kernel trace can be split per leg
(tools/wgrad_stream_trace.py).  Run it with the knob on and off, in fresh processes:

  CESM_WGRAD_STREAM=1 python3 tools/wgrad_stream_legs.py [steps] [legs] [sync]
legs: "AB" (default), "B", ...; sync: "step" (synchronize after every step, per-step times) or "end" (as bench.py:
only after the timed steps, the host free to run ahead -- the average step time is printed).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from cesm_emulator_amd import kernels as K  # noqa: E402
from cesm_emulator_amd.model import Diffusion  # noqa: E402
from cesm_emulator_amd.optim import FusedAdamW  # noqa: E402
from cesm_emulator_amd.train import build_model_from_config, train_step, rank_generator  # noqa: E402

LEGS = {"A": ("more_blocks", 8), "B": ("baseline", 8)}
KEYS = ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams",
        "allocated_bytes.all.peak", "reserved_bytes.all.current")


def leg(name, steps, dev, sync="step"):
    cname, B = LEGS[name]
    cfg = json.load(open(os.path.join(ROOT, "config", cname)))
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    diff.generator = rank_generator(dev, 2, 0)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, max_grad_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(1000)
    x0 = torch.randn(B, 1, 192, 288, device=dev, generator=g)
    cond = torch.randn(B, 1, 12, 192, 288, device=dev, generator=g)
    for _ in range(3):
        train_step(diff, opt, x0, cond, 1.0, None)
    torch.cuda.synchronize()
    s0 = torch.cuda.memory_stats(dev)
    K.call("cesm_hold_cus", 1, 1.0, torch.cuda.current_stream().cuda_stream)  # trace marker
    torch.cuda.synchronize()
    ts = []
    if sync == "step":
        for _ in range(steps):
            t0 = time.perf_counter()
            train_step(diff, opt, x0, cond, 1.0, None)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
    else:
        t0 = time.perf_counter()
        for _ in range(steps):
            train_step(diff, opt, x0, cond, 1.0, None)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3 / steps)
    s1 = torch.cuda.memory_stats(dev)
    d = {k: s1.get(k, 0) - (s0.get(k, 0) if not k.endswith((".peak", ".current")) else 0) for k in KEYS}
    print(f"leg {name} ({cname} B={B}) WGRAD_STREAM={os.environ.get('CESM_WGRAD_STREAM', '0')} sync={sync}: ms/step "
          + " ".join(f"{t:.1f}" for t in ts) + f" | allocator over the timed steps: {d}", flush=True)
    del diff, opt, unet, x0, cond
    torch.cuda.empty_cache()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    legs = sys.argv[2] if len(sys.argv) > 2 else "AB"
    sync = sys.argv[3] if len(sys.argv) > 3 else "step"
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    for name in legs:
        leg(name, steps, dev, sync)


if __name__ == "__main__":
    main()
