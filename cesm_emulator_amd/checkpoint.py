"""Reference-format checkpoints (§8(b) B2).

train.py:1154-1165 (DDP / single-GPU branch) writes
    {"epoch", "model": UNet state_dict, "diffusion_buffers": the 8 schedule buffers,
     "optimizer": torch.optim.AdamW state_dict, "config"}
and train.py:915-946 / inference.py:47-73 read it back.  The UNet / Diffusion here carry the same
state_dict keys and FusedAdamW.state_dict() is in torch.optim.AdamW layout, so a checkpoint written by
either side loads on the other.  Loading uses torch.load(weights_only=True): tensors, numbers and the
JSON config only.
"""
from __future__ import annotations

import torch

from .model import UNet, Diffusion


def save_checkpoint(path, diffusion, optimizer, epoch, config):
    """train.py:1154-1165."""
    full = diffusion.state_dict()
    model_sd = {k[len("model."):]: v for k, v in full.items() if k.startswith("model.")}
    diff_buf = {k: v for k, v in full.items() if not k.startswith("model.")}
    torch.save({"epoch": epoch, "model": model_sd, "diffusion_buffers": diff_buf,
                "optimizer": optimizer.state_dict() if optimizer is not None else {}, "config": config}, path)


def load_checkpoint(ckpt_path, unet, diffusion, optimizer=None, device="cuda"):
    """train.py:915-946: weights (strict=False, missing/unexpected keys reported as the reference does),
    diffusion buffers, optimizer state; returns the epoch to resume at."""
    ckpt = torch.load(ckpt_path, map_location=device, weights_only=True)
    missing, unexpected = unet.load_state_dict(ckpt["model"], strict=False)
    if missing or unexpected:
        print("[UNet] missing keys:", missing)
        print("[UNet] unexpected keys:", unexpected)
    diff_state = diffusion.state_dict()
    diff_state.update(ckpt.get("diffusion_buffers", {}))
    diffusion.load_state_dict(diff_state, strict=False)
    if optimizer is not None and ckpt.get("optimizer"):
        optimizer.load_state_dict(ckpt["optimizer"])
    start_epoch = int(ckpt.get("epoch", 0)) + 1
    print(f"[Resume] Loaded {ckpt_path}. Resuming at epoch {start_epoch}.")
    return start_epoch


def build_from_config(cfg, device):
    """inference.py:25-45 (_build_model_from_ckpt_config)."""
    unet_cfg, train_cfg = cfg.get("unet", {}), cfg.get("train", {})
    unet = UNet(in_channels=unet_cfg.get("in_channels", 2), out_channels=unet_cfg.get("out_channels", 1),
                base_ch=unet_cfg.get("base_ch", 64), ch_mults=tuple(unet_cfg.get("ch_mults", (1, 2, 4))),
                num_res_blocks=unet_cfg.get("num_res_blocks", 2), time_dim=unet_cfg.get("time_dim", 256),
                groups=unet_cfg.get("groups", 8), dropout=unet_cfg.get("dropout", 0.0)).to(device)
    diffusion = Diffusion(unet, img_channels=1, timesteps=train_cfg.get("timesteps", 1000),
                          beta_schedule=train_cfg.get("beta_schedule", "linear")).to(device)
    return unet, diffusion


def load_diffusion_from_checkpoint(ckpt_path, device="cuda"):
    """inference.py:47-73: returns (diffusion in eval mode with frozen parameters, config)."""
    dev = torch.device(device)
    ckpt = torch.load(ckpt_path, map_location=dev, weights_only=True)
    cfg = ckpt.get("config", {})
    unet, diffusion = build_from_config(cfg, dev)
    missing, unexpected = unet.load_state_dict(ckpt["model"], strict=False)
    if missing or unexpected:
        print("[UNet] missing keys:", missing)
        print("[UNet] unexpected keys:", unexpected)
    diff_state = diffusion.state_dict()
    diff_state.update(ckpt.get("diffusion_buffers", {}))
    diffusion.load_state_dict(diff_state, strict=False)
    diffusion.eval()
    for p in diffusion.parameters():
        p.requires_grad_(False)
    return diffusion, cfg
