"""Phase breakdown of tw_bwd from the diagnostic build's in-kernel stamps.
usage: CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_diag.so python tools/tw_stamps.py [emit 0|1]"""
import ctypes
import subprocess
import sys
import os

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from cesm_emulator_amd import _lib  # noqa: E402

sys.argv = [sys.argv[0], "64", "2"] + sys.argv[1:2]
import tblock_micro  # noqa: E402

tblock_micro.main()
n = 4096 * 8
buf = (ctypes.c_ulonglong * n)()
fn = _lib.lib().cesm_diag_tw_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert fn(buf, n) == 0
import numpy as np  # noqa: E402
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.float64)
a = a[a.sum(1) > 0]
names = ["ln+dy load", "qkv (x8 heads)", "dO+bias", "core (4 px)", "dxn+emit", "ln bwd", "-", "-"]
tot = a.sum(1).mean()
print(f"waves {len(a)}, mean cycles per wave {tot:.3e}")
for i in range(6):
    print(f"  {names[i]:16s} {a[:, i].mean():.3e}  {100 * a[:, i].mean() / tot:5.1f} %")
