"""Region bisection of the SLP repeatability defect: run tools/slp_bwd_diff.run on small shapes
with a library whose tblock.hip was built with the SLP vectorizer ON and an empty inline-asm register fence after one
code region of twh_bwd (the fence keeps SLP from packing values across it).  A region whose fence makes the backward
repeatable is where the vectorized code reads registers it did not write.

  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_slpA.so python tools/slp_region_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from slp_bwd_diff import run  # noqa: E402

if __name__ == "__main__":
    print("lib:", os.environ.get("CESM_HIP_LIB", "default"), flush=True)
    dev = torch.device("cuda")
    for (B, H, W) in ((1, 1, 4), (1, 4, 4), (1, 12, 16)):
        run(dev, B, H, W, calls=4)
