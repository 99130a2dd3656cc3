"""Workload for the PMC traffic passes: the bench's training step (same model, batch, window) run for
1 warm-up + `steps` steps, then one device copy of a known byte count for the counter calibration
(tools/step_traffic.py).  Run under rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes).
usage: python tools/step_pmc.py [steps] [batch] [frames] [config]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cesm_emulator_amd.model import Diffusion  # noqa: E402
from cesm_emulator_amd.optim import FusedAdamW  # noqa: E402
from cesm_emulator_amd.train import build_model_from_config, train_step, rank_generator  # noqa: E402

COPY_BYTES = 1 << 30  # past the 256 MiB Infinity Cache


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    F = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    cfg_name = sys.argv[4] if len(sys.argv) > 4 else "more_blocks"
    dev = torch.device("cuda:0")
    cfg = json.load(open(os.path.join(ROOT, "config", cfg_name)))
    torch.manual_seed(1)
    unet = build_model_from_config(cfg["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    diff.generator = rank_generator(dev, 2, 0)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, weight_decay=1e-4, max_grad_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(1000)
    x0 = torch.randn(B, 1, 192, 288, device=dev, generator=g)
    cond = torch.randn(B, 1, F, 192, 288, device=dev, generator=g)
    for _ in range(1 + steps):
        train_step(diff, opt, x0, cond, 1.0, None)
    torch.cuda.synchronize()
    a = torch.empty(COPY_BYTES // 4, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    print(json.dumps({"steps": steps, "batch": B, "frames": F, "config": cfg_name, "copy_bytes": COPY_BYTES}))


if __name__ == "__main__":
    main()
