"""Phase timeline of the halo conv (conv3x3_bf16_kernel<36,7>) from the diagnostic build's in-kernel stamps
(-DCESM_H3_STAMPS, tools/build_diag.sh): per wave, cycles in [end-of-chunk barrier, stage issue, landing wait,
post-landing barrier, MFMA taps, epilogue], and whether the two blocks sharing a CU run their chunks in phase.

usage: DIAG_FLAGS=-DCESM_H3_STAMPS bash tools/build_diag.sh   (in the container)
       CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_diag.so python tools/h3_stamps.py [levels]"""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, ".")
from cesm_emulator_amd import _lib  # noqa: E402
from cesm_emulator_amd import kernels as K  # noqa: E402

# (the s_memtime stamp after the stage's issue already waits for the DMA to land -- see DESIGN §6e -- so "stage" is
# issue + landing and "landing wait" is what is left after it)
NAMES = ["end barrier", "stage issue", "landing wait", "post-land barrier", "MFMA taps", "epilogue"]


def run(lvl, C1=None, Cout=None, Nb=96):
    H, W = 192 >> lvl, 288 >> lvl
    C = 64 << lvl
    C1 = C1 or C
    Cout = Cout or C
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(Nb, H, W, C1, device=dev).to(torch.bfloat16)
    w = torch.randn(Cout, C1, 3, 3, device=dev) * (9 * C1) ** -0.5
    wp = K.conv_pack(w, torch.bfloat16, Cout, C1, 3, 3, 0, 0)
    b = torch.zeros(Cout, device=dev)
    geom = (H, W, Cout, 3, 3, 1, 1, 1)
    lib = _lib.lib()
    setf = lib.cesm_diag_h3_stamps_set
    setf.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(20):  # warm clocks
        K.conv_fwd(x, None, wp, b, geom)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        K.conv_fwd(x, None, wp, b, geom)
    e.record()
    torch.cuda.synchronize()
    us_plain = s.elapsed_time(e) * 1e3 / 10
    nblk = 1 << 16
    buf = torch.zeros(nblk * 4 * 16, dtype=torch.int64, device=dev)
    assert setf(buf.data_ptr(), nblk) == 0
    s.record()
    K.conv_fwd(x, None, wp, b, geom)
    e.record()
    torch.cuda.synchronize()
    assert setf(None, 0) == 0
    us = s.elapsed_time(e) * 1e3
    a = buf.view(-1, 16).cpu().numpy().astype(np.uint64)
    a = a[a[:, 1] > 0]
    hw = a[:, 0]
    t0 = a[:, 1].astype(np.float64)
    t1 = a[:, 2].astype(np.float64)
    ph = a[:, 3:9].astype(np.float64)
    land = a[:, 9:16].astype(np.float64)
    flop = 2.0 * Nb * H * W * Cout * C1 * 9
    nchunk = C1 // 32
    tot = (t1 - t0).mean()
    print(f"level {lvl}: {C1}->{Cout} Nb={Nb} {H}x{W}, {nchunk} chunks: {us_plain:.1f} us plain, {us:.1f} us stamped "
          f"({flop / us_plain / 1e6:.0f} TF/s plain); waves {len(a)}; mean cycles per wave {tot:.0f}")
    for i, nm in enumerate(NAMES):
        per = ph[:, i].mean() / (nchunk if i < 5 else 1)
        print(f"  {nm:18s} {ph[:, i].mean():9.0f} cyc/wave  {100 * ph[:, i].mean() / tot:5.1f} %   {per:7.0f} per chunk")
    # ideal MFMA cycles per chunk and wave: 9 taps x 28 MFMAs x 16 cycles
    print(f"  MFMA issue floor per chunk and wave: {9 * 28 * 16} cyc")
    # co-residency: blocks on the same CU (xcc, se, sh, cu) overlapping in time; wave 0 of each block
    w0 = np.arange(len(a)) % 4 == 0
    key = [(int(h >> 32), int(h >> 8) & 0xFF) for h in hw]
    by_cu = defaultdict(list)
    for i in np.nonzero(w0)[0]:
        by_cu[key[i]].append(i)
    offs = []
    npair = 0
    for cu, idx in by_cu.items():
        idx.sort(key=lambda i: t0[i])
        for p in range(len(idx)):
            for q in range(p + 1, len(idx)):
                i, j = idx[p], idx[q]
                if t0[j] >= t1[i]:
                    break
                npair += 1
                la, lb = land[i][land[i] > 0], land[j][land[j] > 0]
                if len(la) < 3 or len(lb) < 3:
                    continue
                period = np.diff(la).mean()
                for v in lb:
                    if la[0] <= v <= la[-1]:
                        d = np.abs(la - v).min()
                        offs.append(d / period)
    if offs:
        h, _ = np.histogram(offs, bins=5, range=(0, 0.5))
        print(f"  co-resident pairs {npair}; landing offset / chunk period (0 = in phase, 0.5 = alternating): "
              f"mean {np.mean(offs):.2f}, histogram {h.tolist()}")


def main():
    levels = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 3]
    assert "diag" in os.environ.get("CESM_HIP_LIB", ""), "run with CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_diag.so"
    for lvl in levels:
        run(lvl)


if __name__ == "__main__":
    main()
