"""HIP-event time of the optimizer-step weight re-pack (cesm_conv_pack_batch over every cached pack of the more_blocks
UNet, bf16) after one small training step has filled the pack cache.  usage: python tools/pack_time.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from cesm_emulator_amd.config import load_config  # noqa: E402
from cesm_emulator_amd.model import Diffusion  # noqa: E402
from cesm_emulator_amd.optim import FusedAdamW  # noqa: E402
from cesm_emulator_amd.train import build_model_from_config, train_step  # noqa: E402
from tblock_time import timed  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    torch.manual_seed(1)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    unet = build_model_from_config(load_config(os.path.join(root, "config", "more_blocks"))["unet"]).to(dev)
    unet.compute_dtype = torch.bfloat16
    diff = Diffusion(unet).to(dev)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    x0 = torch.randn(1, 1, 32, 48, device=dev)
    cond = torch.randn(1, 1, 12, 32, 48, device=dev)
    train_step(diff, opt, x0, cond, 1.0, None)
    train_step(diff, opt, x0, cond, 1.0, None)
    ex = [m for m in unet.modules() if hasattr(m, "_repack_all")]
    if not ex:
        ex = [v for v in vars(unet).values() if hasattr(v, "_repack_all")]
    e = ex[0]
    n = sum(1 for v in e._pack_cache.values() if v.out.dtype == torch.bfloat16)
    elems = sum(v.out.numel() for v in e._pack_cache.values() if v.out.dtype == torch.bfloat16)
    e._repack_all((-1, -1))  # builds the job table
    tab, nblocks = e._pack_tables[torch.bfloat16]
    from cesm_emulator_amd import kernels as K
    t = timed(lambda: K.conv_pack_batch(tab, n, torch.bfloat16, nblocks), reps)
    print(f"repack of {n} bf16 packs ({elems / 1e6:.1f} M elements, {nblocks} blocks): {t:.1f} us per launch", flush=True)


if __name__ == "__main__":
    main()
