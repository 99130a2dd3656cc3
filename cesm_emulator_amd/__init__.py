"""cesm_emulator_amd — MI355X-native (gfx950) drop-in for the video_net training hot path of
kallenordling/cesm_emulator: `model.UNet` / `model.Diffusion` surface, HIP kernels for every
network op and for the AdamW step, RCCL data parallelism, device-side training-window gather.
"""
from .model import UNet, Diffusion  # noqa: F401
from .optim import FusedAdamW  # noqa: F401

__all__ = ["UNet", "Diffusion", "FusedAdamW"]
