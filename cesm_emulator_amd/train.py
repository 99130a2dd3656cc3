"""Training step / epoch on the HIP path — mirrors train.py:808-911 (train_one_epoch, DDP branch).

Differences from the reference, all deliberate:
  * bf16 kernels instead of fp16 autocast + GradScaler (BASELINE.json asks for bf16; no loss
    scaling is needed) — `use_amp=False` selects the fp32 kernels;
  * the isfinite(loss) guard runs on device (the AdamW kernel skips a non-finite step) and is
    raised on the host when the loss is read, instead of forcing a sync before backward;
  * data-parallel gradient averaging is actually performed (the reference's DDP reducer is never
    armed): bucketed all-reduces overlapped with the backward (`dp.arm` /
    `dp.finish`, distributed.py).
"""
from __future__ import annotations

import torch

from .model import UNet, Diffusion
from .optim import FusedAdamW


def build_model_from_config(cfg_unet):
    """train.py:669-680."""
    return UNet(in_channels=cfg_unet.get("in_channels", 2), out_channels=cfg_unet.get("out_channels", 1),
                base_ch=cfg_unet.get("base_ch", 64), ch_mults=tuple(cfg_unet.get("ch_mults", (1, 2, 4))),
                num_res_blocks=cfg_unet.get("num_res_blocks", 2), time_dim=cfg_unet.get("time_dim", 256),
                groups=cfg_unet.get("groups", 8), use_checkpoint=cfg_unet.get("use_checkpoint", True),
                dropout=cfg_unet.get("dropout", 0.0))


def rank_generator(device, seed=2, rank=0):
    """per-rank t / eps stream for Diffusion.generator: seed + rank (SURVEY.md §8(e) E1 — the reference
    draws from the default generator, model.py:205-206, which is identical on every rank after the same
    manual_seed)."""
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) + int(rank))
    return g


def dp_generator(device, dp, seed=None):
    """the per-rank t / eps stream of a data-parallel run: base seed `seed` (e.g. the training config's), or
    one drawn on rank 0 from the default generator and broadcast, so every rank agrees on it whatever its
    default generator state; the rank is the all-reducer's own (dp.rank), not a global lookup"""
    if seed is None:
        s = torch.randint(0, 2**31 - 1, (1,), dtype=torch.int64)
        if getattr(dp, "world", 1) > 1 and torch.distributed.is_initialized():
            dev = device if torch.distributed.get_backend() == "nccl" else torch.device("cpu")
            s = s.to(dev)
            torch.distributed.broadcast(s, src=0)
        seed = int(s.item())
    return rank_generator(device, seed, getattr(dp, "rank", 0))


def make_optimizer(diffusion, train_cfg):
    """train.py:1077-1083 (+ the clip of :865 folded into the fused step)."""
    opt = train_cfg.get("optimizer", {})
    return FusedAdamW(diffusion.parameters(), lr=opt.get("lr", 2e-4), betas=tuple(opt.get("betas", (0.9, 0.999))),
                      weight_decay=opt.get("weight_decay", 1e-4), max_grad_norm=train_cfg.get("max_grad_norm", 1.0))


def train_step(diffusion, optimizer, x0, cond, max_grad_norm=1.0, dp=None, t=None, noise=None):
    """One optimizer step; returns the loss as a device tensor (no host sync)."""
    optimizer.zero_grad(set_to_none=True)
    net = diffusion.model.net
    overlap = dp is not None and getattr(dp, "overlap", True)
    if overlap:
        dp.arm(net, optimizer.flat)  # bucket all-reduces issued during the backward
    loss = diffusion.loss(x0, cond, t=t, noise=noise)
    loss.backward()
    if overlap:
        dp.finish(net)
    elif dp is not None:
        dp.allreduce_grads(optimizer.flat.grad)
    optimizer.max_grad_norm = max_grad_norm
    optimizer.step(loss=loss.detach())
    return loss.detach()


def train_one_epoch(diffusion, dl, optimizer, device, max_grad_norm=1.0, use_amp=True, epoch=1, dp=None, seed=None):
    """train.py:808-911; returns the epoch's mean loss.  With dp (world > 1) and no generator set yet, each rank
    draws t / eps from its own stream (dp_generator: base `seed`, or one broadcast from rank 0)."""
    diffusion.train()
    diffusion.model.compute_dtype = torch.bfloat16 if use_amp else torch.float32
    if dp is not None and getattr(dp, "world", 1) > 1 and diffusion.generator is None:
        diffusion.generator = dp_generator(device, dp, seed)
    total, steps = 0.0, 0
    for step, (cond, x0) in enumerate(dl, start=1):
        cond = cond.to(device, non_blocking=True)
        x0 = x0.to(device, non_blocking=True)
        loss = train_step(diffusion, optimizer, x0, cond, max_grad_norm, dp)
        val = float(loss.item())
        if not torch.isfinite(torch.tensor(val)):
            raise RuntimeError(f"Non-finite loss at epoch {epoch} step {step}: {val}")
        total += val
        steps += 1
    return total / max(1, steps)
