"""Thin tensor-level wrappers over libcesm_hip.so (one C call each, no torch compute).

Every wrapper takes torch tensors living on the current HIP device, allocates its outputs and
workspaces through the PyTorch caching allocator (plumbing) and enqueues the kernel on
torch's current stream.  Shapes are asserted on the host before launch so a bad call raises
instead of faulting on the GPU.
"""
from __future__ import annotations

import os

import torch

from ._lib import call, lib

F32, BF16 = 0, 1
_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dtcode(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def S():
    return torch.cuda.current_stream().cuda_stream


def P(t):
    return 0 if t is None else t.data_ptr()


def _chk(t, shape=None, dtype=None):
    if t is None:
        return
    if not t.is_cuda:
        raise RuntimeError("cesm_emulator_amd kernels need device tensors (no CPU fallback)")
    if not t.is_contiguous():
        raise RuntimeError("expected a contiguous tensor")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise RuntimeError(f"shape mismatch: got {tuple(t.shape)}, expected {tuple(shape)}")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"dtype mismatch: got {t.dtype}, expected {dtype}")


def empty(shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


# ------------------------------------------------------------------------------------ conv
def conv_pack(w: torch.Tensor, dtype, cout, cin, kh, kw, swap, flip):
    _chk(w, dtype=torch.float32)
    out = empty((cout, kh * kw * cin), dtype, w.device)
    call("cesm_conv_pack", _DT[dtype], P(w), P(out), cout, cin, kh, kw, int(swap), int(flip), S())
    return out


def conv_pack_into(w, out, cout, cin, kh, kw, swap, flip):
    """re-pack into an existing GEMM-layout buffer"""
    _chk(w, dtype=torch.float32)
    call("cesm_conv_pack", _DT[out.dtype], P(w), P(out), cout, cin, kh, kw, int(swap), int(flip), S())
    return out


def pack_blocks(cout, cin, kh, kw):
    """blocks cesm_conv_pack_batch gives one job: (co, ci) tiles of pb_co_t(T) rows x 64 channels (csrc/conv.hip)"""
    T = kh * kw
    cot = min(64, max(1, 4096 // (T * 64)))
    return -(-cout // cot) * -(-cin // 64)


def conv_pack_table(rows, device):
    """device job table of cesm_conv_pack_batch: rows [src ptr, dst ptr, Cout, Cin, KH, KW, swap, flip], then the
    per-job block starts (exclusive prefix of pack_blocks), then the job index of every block; returns (table, nblocks)"""
    assert len(rows) > 0 and all(r[4] * r[5] <= 64 for r in rows)  # a tile's taps x 64 channels fit the LDS tile
    starts, bjob = [0], []
    for j, r in enumerate(rows):
        n = pack_blocks(r[2], r[3], r[4], r[5])
        starts.append(starts[-1] + n)
        bjob += [j] * n
    flat = [v for r in rows for v in r] + starts + bjob
    return torch.tensor(flat, dtype=torch.int64).to(device), starts[-1]


def conv_pack_batch(jobs_dev, njobs, dtype, nblocks):
    """one launch re-packing every job of a conv_pack_table (see cesm_conv_pack_batch)"""
    call("cesm_conv_pack_batch", _DT[dtype], P(jobs_dev), int(njobs), int(nblocks), S())


_QUEUES = {}


def work_queue():
    """the caller-owned int32[2] work counter of the persistent convs' dynamic item claiming (cesm_conv_fwd's queue):
    one per (device, stream) -- launches on one stream run in order, so they share it.  cesm_conv_fwd zeroes it with a
    stream-ordered memset before every launch that uses it (round 6, ADVICE r5: a launch cut short can no longer leave
    a stale count that makes the next one skip its items).  Not allocated during graph capture (the allocation would
    belong to the graph's private pool): a capture that finds no counter for its stream gets the static item split, as
    does CESM_CONV_STATIC=1."""
    if STATIC_CONV:
        return 0
    st = torch.cuda.current_stream()
    key = (st.device.index, st.cuda_stream)
    q = _QUEUES.get(key)
    if q is None:
        if torch.cuda.is_current_stream_capturing():
            return 0
        q = _QUEUES[key] = torch.zeros(4, dtype=torch.int32, device=st.device)
    return q.data_ptr()


STATIC_CONV = os.environ.get("CESM_CONV_STATIC", "0") == "1"


def conv_fwd(x1, x2, wp, bias, geom, res=None, res2=None, out_split=None):
    """geom = (Ho, Wo, Cout, KH, KW, S, P, U).  Returns y (or (y1, y2) when out_split=Co1)."""
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    Nb, Hi, Wi, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    _chk(x1)
    if x2 is not None:
        _chk(x2, (Nb, Hi, Wi, C2), x1.dtype)
    _chk(wp, (Cout, KH * KW * (C1 + C2)), x1.dtype)
    if bias is not None:
        _chk(bias, (Cout,), torch.float32)
    Co1 = Cout if out_split is None else out_split
    y1 = empty((Nb, Ho, Wo, Co1), x1.dtype, x1.device)
    y2 = empty((Nb, Ho, Wo, Cout - Co1), x1.dtype, x1.device) if Co1 != Cout else None
    _chk(res, (Nb, Ho, Wo, Co1), x1.dtype)
    _chk(res2, (Nb, Ho, Wo, Cout - Co1), x1.dtype)
    call("cesm_conv_fwd", dtcode(x1), P(x1), P(x2), P(wp), P(bias), P(res), P(res2), P(y1), P(y2), Nb, Hi, Wi, C1,
         C2, Ho, Wo, Cout, Co1, KH, KW, St, Pd, U, work_queue(), S())
    if CONV_TRACE is not None:
        CONV_TRACE.append(("fwd", Nb, Hi, Wi, C1 + C2, Ho, Wo, Cout, KH, KW, St, Pd, U))
    return y1 if y2 is None else (y1, y2)


def conv_gn_nslot(x1, x2, geom, B):
    """GroupNorm partial slots per sample cesm_conv_fwd_gn writes for this conv (0: the kernel has none)"""
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    Nb, Hi, Wi, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    return int(lib().cesm_conv_gn_nslot(dtcode(x1), Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, KH, KW, St, Pd, U, B))


def conv_fwd_gn(x1, x2, wp, bias, geom, B, nslot):
    """conv_fwd of a Block conv (video_net.py:215) that also writes the GroupNorm statistics partials of its
    output (per sample, slot and channel quad: sum, sum of squares); returns (y, part) for gn_stats_part"""
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    Nb, Hi, Wi, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    _chk(x1)
    if x2 is not None:
        _chk(x2, (Nb, Hi, Wi, C2), x1.dtype)
    _chk(wp, (Cout, KH * KW * (C1 + C2)), x1.dtype)
    if bias is not None:
        _chk(bias, (Cout,), torch.float32)
    y = empty((Nb, Ho, Wo, Cout), x1.dtype, x1.device)
    part = empty((B, nslot, Cout // 4, 2), torch.float32, x1.device)
    call("cesm_conv_fwd_gn", dtcode(x1), P(x1), P(x2), P(wp), P(bias), P(y), P(part), B, Nb, Hi, Wi, C1, C2, Ho, Wo,
         Cout, KH, KW, St, Pd, U, work_queue(), S())
    if CONV_TRACE is not None:
        CONV_TRACE.append(("fwd", Nb, Hi, Wi, C1 + C2, Ho, Wo, Cout, KH, KW, St, Pd, U))
    return y, part


def qkv_bwd_supported(M, C):
    return lib().cesm_qkv_bwd_streams(int(M), 768, int(C)) > 0


def qkv_bwd(dy, x, wt, dw, accumulate=True):
    """backward of the 768-channel qkv projection, dqkv read once (csrc/qkvbwd.hip): returns dx [..., C] (the LN
    output's gradient); dw [768, C] fp32 (+)= dy^T x (nullable).  dy [..., 768], x [..., C] bf16 with the same rows;
    wt [C, 768] bf16 = the weight transposed (conv_pack(w, bf16, C, 768, 1, 1, 1, 1))."""
    C = x.shape[-1]
    M = x.numel() // C
    _chk(x, dtype=torch.bfloat16)
    _chk(dy, dtype=torch.bfloat16)
    _chk(wt, (C, 768), torch.bfloat16)
    if dy.numel() != M * 768:
        raise RuntimeError(f"qkv_bwd: dy has {dy.numel()} elements, expected {M} x 768")
    ns = lib().cesm_qkv_bwd_streams(M, 768, C)
    if ns <= 0:
        raise ValueError(f"qkv_bwd: unsupported shape M={M} C={C}")
    dev = x.device
    dx = empty(x.shape, torch.bfloat16, dev)
    slab = None
    if dw is not None:
        _chk(dw, dtype=torch.float32)
        if dw.numel() != 768 * C:
            raise RuntimeError("qkv_bwd: dw must hold 768 x C floats")
        slab = empty(((C // 64) * ns * 768 * 64,), torch.float32, dev)
    call("cesm_qkv_bwd", P(dy), P(x), P(wt), P(dx), P(dw), P(slab), M, 768, C, int(accumulate), S())
    return dx


# shape log of conv launches (set CESM_TRACE_CONV=1; tools/conv_shapes.py prints it)
CONV_TRACE = [] if os.environ.get("CESM_TRACE_CONV") else None


# target block count of the split-K weight-gradient launches: every split writes a full fp32
# [Cout][K] slab that conv_wgrad_reduce reads back, so more blocks than ~2-4 per CU only adds slab
# traffic (round 3: 512 / 2048 blocks 144.7 / 131.2 ms per step against 129.7 at 1024)
WGRAD_BLOCKS = 1024
# blocks of the square-tile 1x1 weight-gradient kernel (512 threads, 64 KB of LDS: two per CU)
WGRAD_SQ_BLOCKS = 256


def _wgrad_nsplit(M, cout, K, bm=64, blocks=None):
    """pixel splits of the weight-gradient GEMM: ~`blocks` blocks of (bm x 64) tiles, >= 256 pixels each"""
    tiles = max(1, cout // bm) * max(1, K // 64)
    n = max(1, (blocks or WGRAD_BLOCKS) // tiles)
    n = min(n, max(1, M // 256))
    return n


def _wgrad_bm(x, cout, co1):
    if x.dtype != torch.bfloat16:
        return 64
    if cout % 256 == 0 and co1 % 256 == 0:
        return 256
    if cout % 128 == 0 and co1 % 128 == 0:
        return 128
    return 64


def conv_wgrad(x1, x2, dy1, dy2, dw, geom, swap, flip, accumulate=True, db=None):
    """dW of a conv (split-K over pixels + reduce).  db: also the bias gradient (+=) in the same pass when
    the bf16 wide-tile kernel runs; returns True if db was produced (else the caller runs colsum)."""
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    Nb, Hi, Wi, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    Co1 = dy1.shape[3]
    _chk(dy1, (Nb, Ho, Wo, Co1), x1.dtype)
    _chk(dy2, None if dy2 is None else (Nb, Ho, Wo, Cout - Co1), x1.dtype)
    _chk(dw, dtype=torch.float32)
    K = KH * KW * (C1 + C2)
    M = Nb * Ho * Wo
    halo3 = KH == 3 and KW == 3 and St == 1 and Pd == 1 and U == 1
    # 4x4 stride-2 (Downsample / the Upsample's weight gradient): wgrads2 kernel, blocks of 64 co x 32 ci x one
    # input parity (4 taps); its bias gradient is the caller's column sum (same condition as cesm_conv_wgrad)
    s2 = (KH == 4 and KW == 4 and St == 2 and Pd == 1 and U == 1 and Hi == 2 * Ho and Wi == 2 * Wo and Wo >= 64
          and x2 is None
          and dy2 is None and x1.dtype == torch.bfloat16)
    if (halo3 or s2) and x1.dtype == torch.bfloat16:
        # halo wgrad kernels: blocks of 64 co x 32 ci (all 9 taps / one parity's 4), split over pixel tiles
        nb = WGRAD_BLOCKS // 2
        nsplit = max(1, min(nb // max(1, (Cout // 64) * ((C1 + C2) // 32) * (4 if s2 else 1)), max(1, M // 256)))
    else:
        sq = lib().cesm_conv_wgrad_sq_bn(dtcode(x1), Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, St, Pd, U,
                                         int(db is not None))
        if sq:
            # square-tile 1x1 kernel: 512-thread blocks of 256 (or 64) x sq, ~WGRAD_SQ_BLOCKS of them (twice as many
            # 64-row blocks: 100 registers, two per CU)
            nb = WGRAD_SQ_BLOCKS * (2 if Cout == 64 else 1)
            nsplit = max(1, min(nb // (max(1, Cout // 256) * (K // sq)), max(1, M // 256)))
        else:
            bm = _wgrad_bm(x1, Cout, Co1)
            nsplit = _wgrad_nsplit(M, Cout, K, bm, WGRAD_BLOCKS // 2 if bm == 256 else WGRAD_BLOCKS)
    slab = empty((nsplit, Cout, K), torch.float32, x1.device)
    if CONV_TRACE is not None:
        CONV_TRACE.append(("wgrad", Nb, Hi, Wi, C1 + C2, Ho, Wo, Cout, KH, KW, St, Pd, U))
    # the bias rides on the wide-tile kernel only (same dispatch condition as cesm_conv_wgrad)
    wide = x1.dtype == torch.bfloat16 and not halo3 and not s2 and M < (1 << 31) and dy2 is None
    if db is not None and wide:
        _chk(db, (Cout,), torch.float32)
        bslab = empty((nsplit, Cout), torch.float32, x1.device)
    else:
        db = bslab = None
    call("cesm_conv_wgrad", dtcode(x1), P(x1), P(x2), P(dy1), P(dy2), P(dw), P(slab), P(db), P(bslab), nsplit, Nb,
         Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, St, Pd, U, int(swap), int(flip), int(accumulate), S())
    return db is not None



def colsum(x, dst, accumulate=True):
    C = x.shape[-1]
    rows = x.numel() // C
    nsplit = int(max(1, min(1024, rows // 512)))
    part = empty((nsplit, C), torch.float32, x.device)
    call("cesm_colsum", dtcode(x), P(x), P(dst), P(part), nsplit, rows, C, int(accumulate), S())


def stem_fwd(xt, cond, w, b, F, dtype):
    B, Fx, H, W = xt.shape
    Fc = cond.shape[1]
    Co, _, _, KS, _ = w.shape
    _chk(xt, dtype=torch.float32)
    _chk(cond, (B, Fc, H, W), torch.float32)
    y = empty((B * F, H, W, Co), dtype, xt.device)
    call("cesm_stem_fwd", _DT[dtype], P(xt), P(cond), P(w), P(b), P(y), B, F, Fx, Fc, H, W, Co, KS, S())
    return y


def stem_wgrad(xt, cond, dy, dw, F, accumulate=True):
    B, Fx, H, W = xt.shape
    Fc = cond.shape[1]
    Co = dy.shape[3]
    KS = dw.shape[-1]
    nblk = 512
    part = empty((nblk, Co * 2 * KS * KS), torch.float32, xt.device)
    call("cesm_stem_wgrad", dtcode(dy), P(xt), P(cond), P(dy), P(dw), P(part), nblk, B, F, Fx, Fc, H, W, Co, KS,
         int(accumulate), S())


def head_fwd(x, w, b, B, F):
    Nb, H, W, C = x.shape
    out = empty((B, 1, H, W), torch.float32, x.device)
    call("cesm_head_fwd", dtcode(x), P(x), P(w), P(b), P(out), B, F, H * W, C, S())
    return out


def head_bwd(dout, x, w, dw, db, B, F, need_dx=True, accumulate=True):
    Nb, H, W, C = x.shape
    dx = empty(x.shape, x.dtype, x.device) if need_dx else None
    nblk = 256
    part = empty((nblk, C + 1), torch.float32, x.device)
    call("cesm_head_bwd", dtcode(x), P(dout), P(x), P(w), P(dx), P(dw), P(db), P(part), nblk, B, F, H * W, C,
         int(accumulate), S())
    return dx


# ------------------------------------------------------------------------------------ norms
def gn_stats(y, B, G, eps=1e-5):
    C = y.shape[-1]
    rows_b = y.numel() // (C * B)
    stats = empty((B, G, 2), torch.float32, y.device)
    ws = empty((max(B * 256, 1024) * G * 2,), torch.float64, y.device)
    call("cesm_gn_stats", dtcode(y), P(y), P(stats), P(ws), B, rows_b, C, G, float(eps), S())
    return stats


def gn_stats_part(part, rows_b, G, eps=1e-5):
    """GroupNorm (mean, rstd) [B][G][2] from conv_fwd_gn's partials (replaces gn_stats' pass over y)"""
    B, nslot, nq, _ = part.shape
    stats = empty((B, G, 2), torch.float32, part.device)
    call("cesm_gn_stats_part", P(part), P(stats), B, nslot, nq * 4, G, rows_b, float(eps), S())
    return stats


def gn_apply(y, stats, gamma, beta, ss, res, B, G):
    C = y.shape[-1]
    rows_b = y.numel() // (C * B)
    out = empty(y.shape, y.dtype, y.device)
    _chk(res, y.shape, y.dtype)
    ws = empty((2 * B * C,), torch.float32, y.device)
    call("cesm_gn_apply", dtcode(y), P(y), P(stats), P(gamma), P(beta), P(ss), P(res), P(out), P(ws), B, rows_b, C,
         G, S())
    return out


def gn_bwd(dout, y, stats, gamma, beta, ss, dgamma, dbeta, B, G, want_dss, dbias=None):
    """GroupNorm(+scale/shift, SiLU) backward; dbias (+)= sum of dy over rows (the producing conv's bias)"""
    C = y.shape[-1]
    rows_b = y.numel() // (C * B)
    dy = empty(y.shape, y.dtype, y.device)
    dss = empty((B, 2 * C), torch.float32, y.device) if want_dss else None
    ws = empty((max(B * 1024, 1024) * C * 3 + B * C * 3 + B * C * 5,), torch.float32, y.device)  # <= 1024 chunks/sample
    call("cesm_gn_bwd", dtcode(y), P(dout), P(y), P(stats), P(gamma), P(beta), P(ss), P(dy), P(dss), P(dgamma),
         P(dbeta), P(dbias), P(ws), B, rows_b, C, G, 1, S())
    return dy, dss


def ln_fwd(x, gamma, save=True, eps=1e-5, perm=None):
    """perm = (F, HW): write the output rows of voxel (b, f, p) at (b, p, f) -- pixel-major, a pixel's frames
    adjacent (mr stays in x's order)"""
    C = x.shape[-1]
    V = x.numel() // C
    out = empty(x.shape, x.dtype, x.device)
    mr = empty((V, 2), torch.float32, x.device) if save else None
    pf, phw = perm if perm else (0, 0)
    call("cesm_ln_fwd", dtcode(x), P(x), P(gamma), P(out), P(mr), V, C, float(eps), pf, phw, S())
    return out, mr


def ln_bwd(dy, x, mr, gamma, dgamma, dres=None, perm=None):
    """perm = (F, HW): dy rows are pixel-major (as ln_fwd(perm=...) wrote the output); x, dres, dx in x's order"""
    C = x.shape[-1]
    V = x.numel() // C
    dx = empty(x.shape, x.dtype, x.device)
    nblk = 1024
    part = empty((nblk, C), torch.float32, x.device)
    _chk(dres, x.shape, x.dtype)
    pf, phw = perm if perm else (0, 0)
    call("cesm_ln_bwd", dtcode(x), P(dy), P(x), P(mr), P(gamma), P(dres), P(dx), P(dgamma), P(part), nblk, V, C, 1,
         pf, phw, S())
    return dx


def add(a, b):
    out = empty(a.shape, a.dtype, a.device)
    _chk(b, a.shape, a.dtype)
    call("cesm_add", dtcode(a), P(a), P(b), P(out), a.numel(), S())
    return out


# ------------------------------------------------------------------------------------ attention
def rope_table(freqs, F):
    rot = empty((F, 16, 2), torch.float32, freqs.device)
    call("cesm_rope_table", P(freqs), P(rot), F, S())
    return rot


def relpos_fwd(table, F, num_buckets=32, max_distance=32):
    nb, heads = table.shape
    bias = empty((heads, F, F), torch.float32, table.device)
    call("cesm_relpos_fwd", P(table), P(bias), F, heads, num_buckets, max_distance, S())
    return bias


# bf16 temporal-attention core on MFMA (csrc/tflash.hip) for F <= 128; fp32 (parity mode): the VALU kernels
def _tflash(qkv, F):
    return qkv.dtype == torch.bfloat16 and lib().cesm_tflash_supported(F) == 1


def tattn_fwd(qkv, bias, rot, B, F, HW, scale, save=True, pixel_major=False):
    """pixel_major (MFMA core, F > 16): qkv rows ordered [B][HW][F]; out stays [B][F][HW]"""
    V = qkv.shape[0]
    _chk(qkv, (B * F * HW, 768))
    out = empty((V, 256), qkv.dtype, qkv.device)
    lse = empty((B, 8, HW, F), torch.float32, qkv.device) if save else None
    if _tflash(qkv, F):
        call("cesm_tflash_fwd", P(qkv), P(bias), P(rot), P(out), P(lse), B, F, HW, float(scale), int(pixel_major), S())
        return out, lse
    if pixel_major:
        raise ValueError("pixel-major qkv needs the MFMA temporal core (bf16, F <= 128)")
    call("cesm_tattn_fwd", dtcode(qkv), P(qkv), P(bias), P(rot), P(out), P(lse), B, F, HW, float(scale), S())
    return out, lse


def tattn_bwd(qkv, o, dout, lse, bias, rot, dtable, B, F, HW, scale, num_buckets=32, max_distance=32,
              pixel_major=False):
    """pixel_major: qkv and the returned dqkv in [B][HW][F] row order (o, dout frame-major)"""
    dqkv = empty(qkv.shape, qkv.dtype, qkv.device)
    if _tflash(qkv, F):
        _chk(o, (qkv.shape[0], 256), qkv.dtype)
        _chk(dout, (qkv.shape[0], 256), qkv.dtype)
        dev = qkv.device
        nblk = lib().cesm_tflash_nblk(HW)
        dbuf = empty((B, 8, HW, F), torch.float32, dev)
        part = empty((B * 8 * nblk * (2 * F - 1),), torch.float32, dev)
        off = empty((8 * (2 * F - 1),), torch.float32, dev)
        call("cesm_tflash_bwd", P(qkv), P(o), P(dout), P(lse), P(bias), P(rot), P(dqkv), P(dtable), P(dbuf), P(part),
             P(off), B, F, HW, float(scale), num_buckets, max_distance, 1, int(pixel_major), S())
        return dqkv
    if pixel_major:
        raise ValueError("pixel-major qkv needs the MFMA temporal core (bf16, F <= 128)")
    nblk = lib().cesm_tattn_nblk(F, HW)
    part = empty((B * 8 * nblk, F, F), torch.float32, qkv.device)
    call("cesm_tattn_bwd", dtcode(qkv), P(qkv), P(o), P(dout), P(lse), P(bias), P(rot), P(dqkv), P(part), B, F, HW,
         float(scale), S())
    if dtable is not None:
        ws = empty((8, F, F), torch.float32, qkv.device)
        call("cesm_relpos_bwd", P(part), nblk, B, P(dtable), P(ws), F, 8, num_buckets, max_distance, 1, S())
    return dqkv


TBLOCK_C = (64, 128, 256, 512)


def tblock_fwd(x, gamma, wqkv, wout, bias, rot, B, F, scale, save=True, eps=1e-5, save_o=False):
    """fused temporal-attention block forward (bf16); x [B*F, H, W, C].  Returns (y, mr, lse, o); o (the
    attention output before to_out, [B*F, H, W, 256]) only with save_o (C <= 256), for the to_out weight
    gradient, so the backward need not emit it."""
    Nb, H, W, C = x.shape
    _chk(x, dtype=torch.bfloat16)
    _chk(wqkv, (768, C), torch.bfloat16)
    _chk(wout, (C, 256), torch.bfloat16)
    y = empty(x.shape, x.dtype, x.device)
    mr = empty((Nb * H * W, 2), torch.float32, x.device) if save else None
    lse = empty((B, 8, H * W, F), torch.float32, x.device) if save else None
    o = empty((Nb, H, W, 256), x.dtype, x.device) if save_o else None
    wimg = empty(((768 + 256) * C,), torch.bfloat16, x.device)  # weight fragment images (rebuilt per call)
    call("cesm_tblock_fwd", P(x), P(gamma), P(wqkv), P(wout), P(bias), P(rot), P(y), P(mr), P(lse), P(o), P(wimg),
         B, F, H * W, C, float(scale), float(eps), S())
    return y, mr, lse, o


def tblock_bwd(x, dy, gamma, mr, lse, wqkv, wqkv_t, wout_t, bias, rot, dgamma, dtable, B, F, scale,
               want_wgrad_inputs=True, num_buckets=32, max_distance=32, emit_o=True):
    """fused temporal-attention block backward, dx path (bf16).  Returns (dx, dqkv, o, xn); the last
    three ([.., 768], [.., 256], [.., C] bf16) feed the to_qkv / to_out weight-gradient GEMMs."""
    Nb, H, W, C = x.shape
    HW = H * W
    _chk(x, dtype=torch.bfloat16)
    _chk(dy, x.shape, torch.bfloat16)
    _chk(wqkv, (768, C), torch.bfloat16)
    _chk(wqkv_t, (C, 768), torch.bfloat16)
    _chk(wout_t, (256, C), torch.bfloat16)
    if Nb != B * F or mr.shape != (Nb * HW, 2) or lse.shape != (B, 8, HW, F):
        raise ValueError("tblock_bwd: saved statistics do not match x")
    dev = x.device
    dx = empty(x.shape, x.dtype, dev)
    if want_wgrad_inputs:
        dqkv = empty((Nb, H, W, 768), x.dtype, dev)
        o = empty((Nb, H, W, 256), x.dtype, dev) if emit_o else None
        xn = empty(x.shape, x.dtype, dev)
    else:
        dqkv = o = xn = None
    nblk = lib().cesm_tblock_bwd_nblk(B, F, HW, C)
    dbp = empty((B, 8, nblk, F, F), torch.float32, dev)
    dgp = empty((B * nblk, C), torch.float32, dev)
    wimg = empty(((2 * 768 + 256) * C,), torch.bfloat16, dev)  # weight fragment images (rebuilt per call)
    call("cesm_tblock_bwd", P(x), P(dy), P(gamma), P(mr), P(lse), P(wqkv), P(wqkv_t), P(wout_t), P(bias), P(rot),
         P(dx), P(dqkv), P(o), P(xn), P(dbp), P(dgamma), P(dgp), P(wimg), nblk, B, F, HW, C, float(scale), 1, S())
    if dtable is not None:
        ws = empty((8, F, F), torch.float32, dev)
        call("cesm_relpos_bwd", P(dbp), nblk, B, P(dtable), P(ws), F, 8, num_buckets, max_distance, 1, S())
    return dx, dqkv, o, xn


def tblock_bwd_dw_supported(B, F, HW, C):
    """shapes the head-parallel fused backward with in-kernel weight gradients handles (C = 64, 4F <= 48)"""
    return lib().cesm_tblock_bwd_dw_nblk(B, F, HW, C) > 0


def tblock_fwd_fold(x, gamma, wqkv_f32, wout, bias, rot, B, F, scale, save=True, eps=1e-5, save_o=False):
    """tblock_fwd with the LN gamma folded into the QKV weights (the forward of tblock_bwd_dw); wqkv_f32 is
    the fp32 master to_qkv weight [768, C].  Returns (y, mr, lse, o) as tblock_fwd."""
    Nb, H, W, C = x.shape
    _chk(x, dtype=torch.bfloat16)
    _chk(wqkv_f32, (768, C), torch.float32)
    _chk(wout, (C, 256), torch.bfloat16)
    _chk(gamma, (C,), torch.float32)
    y = empty(x.shape, x.dtype, x.device)
    mr = empty((Nb * H * W, 2), torch.float32, x.device) if save else None
    lse = empty((B, 8, H * W, F), torch.float32, x.device) if save else None
    o = empty((Nb, H, W, 256), x.dtype, x.device) if save_o else None
    wimg = empty(((768 + 256) * C,), torch.bfloat16, x.device)
    call("cesm_tblock_fwd_fold", P(x), P(gamma), P(wqkv_f32), P(wout), P(bias), P(rot), P(y), P(mr), P(lse), P(o),
         P(wimg), B, F, H * W, C, float(scale), float(eps), S())
    return y, mr, lse, o


def tblock_bwd_dw(x, dy, mr, lse, wqkv_f32, gamma, wout_t, bias, rot, dwqkv, dgamma, dtable, B, F, scale,
                  num_buckets=32, max_distance=32, emit_o=False):
    """head-parallel fused temporal-block backward with in-kernel weight gradients (C = 64, 4F <= 48):
    returns dx, or (dx, o) with emit_o -- o [Nb, H, W, 256] the attention output recomputed from the backward's P,
    the to_out weight gradient's input (the forward then writes none); dwqkv (+)= the to_qkv weight gradient,
    dgamma (+)= the LN gamma gradient, dtable (+)= the rel-pos table gradient (each nullable).  The forward must
    be tblock_fwd_fold's."""
    Nb, H, W, C = x.shape
    HW = H * W
    _chk(x, dtype=torch.bfloat16)
    _chk(dy, x.shape, torch.bfloat16)
    _chk(wqkv_f32, (768, C), torch.float32)
    _chk(gamma, (C,), torch.float32)
    _chk(wout_t, (256, C), torch.bfloat16)
    _chk(dwqkv, (768, C), torch.float32)
    _chk(dgamma, (C,), torch.float32)
    if Nb != B * F or mr.shape != (Nb * HW, 2) or lse.shape != (B, 8, HW, F):
        raise ValueError("tblock_bwd_dw: saved statistics do not match x")
    nblk = lib().cesm_tblock_bwd_dw_nblk(B, F, HW, C)
    if nblk <= 0:
        raise ValueError(f"tblock_bwd_dw: unsupported shape C={C} F={F}")
    dev = x.device
    dx = empty(x.shape, x.dtype, dev)
    o = empty((Nb, H, W, 256), x.dtype, dev) if emit_o else None
    dbp = empty((8, nblk, F, F), torch.float32, dev)
    slab = empty((nblk * 768 * C,), torch.float32, dev)
    tmp = empty((768, C), torch.float32, dev)
    wimg = empty(((2 * 768 + 256) * C,), torch.bfloat16, dev)
    call("cesm_tblock_bwd_dw", P(x), P(dy), P(mr), P(lse), P(wqkv_f32), P(gamma), P(wout_t), P(bias), P(rot), P(dx),
         P(o), P(dwqkv), P(dgamma), P(dbp), P(slab), P(tmp), P(wimg), nblk, B, F, HW, C, float(scale), 1, S())
    if dtable is not None:
        ws = empty((8, F, F), torch.float32, dev)
        call("cesm_relpos_bwd", P(dbp), nblk, 1, P(dtable), P(ws), F, 8, num_buckets, max_distance, 1, S())
    return (dx, o) if emit_o else dx


# fused SLA at C = 64 and 128 (measured +0.8 % step throughput for C = 128 with the parallel context
# combine)
SLAF_C = (64, 128)


def slaf_fwd(x, gamma, wqkv, wout, bout, scale, eps=1e-5, save_o=False):
    """fused spatial-linear-attention block forward (bf16, C=64/128); x [Nf, H, W, C].
    Returns y and the saved state (mz, ctx32, actT, actx, o) for slaf_bwd; o (the attention output before
    to_out, [Nf, H, W, 256]) only with save_o, for the to_out weight gradient."""
    Nf, H, W, C = x.shape
    HW = H * W
    _chk(x, dtype=torch.bfloat16)
    _chk(wqkv, (768, C), torch.bfloat16)
    _chk(wout, (C, 256), torch.bfloat16)
    dev = x.device
    y = empty(x.shape, x.dtype, dev)
    mz = empty((Nf, 8, 32, 2), torch.float32, dev)
    ctx32 = empty((Nf, 8, 32, 32), torch.float32, dev)
    actT = empty((Nf, 8, 2, 64, 8), torch.bfloat16, dev)
    actx = empty((Nf, 8, 2, 64, 8), torch.bfloat16, dev)
    nblk = lib().cesm_slaf_nblk(Nf, HW)
    ws = empty((nblk * Nf * 8 * 1088,), torch.float32, dev)
    o = empty((Nf, H, W, 256), x.dtype, dev) if save_o else None
    call("cesm_slaf_fwd", P(x), P(gamma), P(wqkv), P(wout), P(bout), P(y), P(o), P(mz), P(ctx32), P(actT), P(actx),
         P(ws), Nf, HW, C, float(scale), float(eps), S())
    return y, (mz, ctx32, actT, actx, o)


def slaf_bwd(x, dy, gamma, wqkv, wqkv_t, wout_t, state, dgamma, scale, want_wgrad_inputs=True, eps=1e-5):
    """fused SLA block backward, dx path (bf16, C=64).  Returns (dx, dqkv, o, xn); the last three feed the
    to_qkv / to_out weight-gradient GEMMs.  When the forward saved o (slaf_fwd save_o), that o is returned
    and the backward does not emit it."""
    Nf, H, W, C = x.shape
    HW = H * W
    mz, ctx32, actT, actx, o_fwd = state
    _chk(dy, x.shape, torch.bfloat16)
    _chk(wqkv_t, (C, 768), torch.bfloat16)
    _chk(wout_t, (256, C), torch.bfloat16)
    dev = x.device
    dx = empty(x.shape, x.dtype, dev)
    if want_wgrad_inputs:
        dqkv = empty((Nf, H, W, 768), x.dtype, dev)
        o = empty((Nf, H, W, 256), x.dtype, dev) if o_fwd is None else None
        xn = empty(x.shape, x.dtype, dev)
    else:
        dqkv = o = xn = None
    nblk = lib().cesm_slaf_nblk(Nf, HW)
    part = empty((nblk * Nf * 8 * 1024,), torch.float32, dev)
    G = empty((Nf, 8, 64, 16), torch.float32, dev)  # per-lane k-softmax offsets + G image
    adc = empty((Nf, 8, 2, 64, 8), torch.bfloat16, dev)
    adcT = empty((Nf, 8, 2, 64, 8), torch.bfloat16, dev)
    dgp = empty((lib().cesm_slaf_bwd_nblk(Nf, HW, C), C), torch.float32, dev)
    wimg = empty(((2 * 768 + 256) * C,), torch.bfloat16, dev)
    call("cesm_slaf_bwd", P(x), P(dy), P(gamma), P(wqkv), P(wqkv_t), P(wout_t), P(mz), P(ctx32), P(actT), P(actx),
         P(dx), P(dqkv), P(o), P(xn), P(dgamma), P(part), P(G), P(adc), P(adcT), P(dgp), P(wimg), Nf, HW, C,
         float(scale), float(eps), 1, S())
    if want_wgrad_inputs and o_fwd is not None:
        o = o_fwd
    return dx, dqkv, o, xn


def pack_scaled(w, colscale, trans=False):
    """bf16 copy of w diag(colscale) (w fp32 [M, K]); trans: the transposed [K, M] layout"""
    M, K = w.shape
    _chk(w, dtype=torch.float32)
    _chk(colscale, (K,), torch.float32)
    out = empty((K, M) if trans else (M, K), torch.bfloat16, w.device)
    call("cesm_pack_scaled", P(w), P(colscale), P(out), M, K, int(trans), S())
    return out


def slaf_bwd_dw_supported(Nf, HW, C):
    return lib().cesm_slaf_bwd_dw_nblk(Nf, HW, C) > 0


def slaf_bwd_dw(x, dy, gamma_one, wq_fold, wqkv_f32, gamma, wout_t, state, dwqkv, dgamma, scale, eps=1e-5,
                dwout=None, dbout=None):
    """fused SLA block backward with in-kernel weight gradients (C = 64); the forward must have been
    slaf_fwd(x, gamma_one, wq_fold, ...) with wq_fold = pack_scaled(wqkv_f32, gamma).  Returns dx; dwqkv /
    dgamma (+)= the to_qkv / LN gamma gradients, dwout [C, 256] / dbout [C] (+)= the to_out weight / bias
    gradients (both or neither; computed from the recomputed q~ and the saved context: no O needed)."""
    Nf, H, W, C = x.shape
    HW = H * W
    mz, ctx32, actT, actx, _o = state
    _chk(x, dtype=torch.bfloat16)
    _chk(dy, x.shape, torch.bfloat16)
    _chk(wq_fold, (768, C), torch.bfloat16)
    _chk(wqkv_f32, (768, C), torch.float32)
    _chk(gamma, (C,), torch.float32)
    _chk(gamma_one, (C,), torch.float32)
    _chk(wout_t, (256, C), torch.bfloat16)
    _chk(dwqkv, (768, C), torch.float32)
    _chk(dgamma, (C,), torch.float32)
    nblk_dx = lib().cesm_slaf_bwd_dw_nblk(Nf, HW, C)
    if nblk_dx <= 0:
        raise ValueError(f"slaf_bwd_dw: unsupported shape C={C}")
    dev = x.device
    dx = empty(x.shape, x.dtype, dev)
    nblk = lib().cesm_slaf_nblk(Nf, HW)
    part = empty((nblk * Nf * 8 * 1024,), torch.float32, dev)
    G = empty((Nf, 8, 64, 16), torch.float32, dev)
    adc = empty((Nf, 8, 2, 64, 8), torch.bfloat16, dev)
    adcT = empty((Nf, 8, 2, 64, 8), torch.bfloat16, dev)
    slab = empty((nblk_dx, 768, C), torch.float32, dev)
    tmp = empty((768, C), torch.float32, dev)
    wimg = empty(((2 * 768 + 256) * C,), torch.bfloat16, dev)
    if (dwout is None) != (dbout is None):
        raise ValueError("slaf_bwd_dw: dwout and dbout go together")
    partm = partb = None
    if dwout is not None:
        _chk(dwout, (C, 256), torch.float32)
        _chk(dbout, (C,), torch.float32)
        partm = empty(((nblk + 1) * Nf * 8 * 2048,), torch.float32, dev)
        partb = empty((nblk * Nf * C,), torch.float32, dev)
    call("cesm_slaf_bwd_dw", P(x), P(dy), P(gamma_one), P(wq_fold), P(wqkv_f32), P(gamma), P(wout_t), P(mz), P(ctx32),
         P(actT), P(actx), P(dx), P(dwqkv), P(dgamma), P(dwout), P(dbout), P(part), P(G), P(adc), P(adcT), P(slab),
         P(tmp), P(partm), P(partb), P(wimg), nblk_dx, Nf, HW, C, float(scale), float(eps), 1, S())
    return dx


def sla_fwd(qkv, Nf, HW, scale):
    nchunk = lib().cesm_sla_nchunk(HW)
    out = empty((qkv.shape[0], 256), qkv.dtype, qkv.device)
    ctx = empty((Nf, 8, 32, 32), torch.float32, qkv.device)
    ml = empty((Nf, 8, 32, 2), torch.float32, qkv.device)
    ws = empty((Nf * 8 * nchunk * (32 + 32 + 1024),), torch.float32, qkv.device)
    call("cesm_sla_fwd", dtcode(qkv), P(qkv), P(out), P(ctx), P(ml), P(ws), Nf, HW, float(scale), S())
    return out, ctx, ml


def sla_bwd(qkv, dout, ctx, ml, Nf, HW, scale):
    nchunk = lib().cesm_sla_nchunk(HW)
    dqkv = empty(qkv.shape, qkv.dtype, qkv.device)
    ws = empty((Nf * 8 * nchunk * 1024 + Nf * 8 * (1024 + 32),), torch.float32, qkv.device)
    call("cesm_sla_bwd", dtcode(qkv), P(qkv), P(dout), P(ctx), P(ml), P(dqkv), P(ws), Nf, HW, float(scale), S())
    return dqkv


# ------------------------------------------------------------------------------------ misc
def sinusoidal(t, dim):
    emb = empty((t.shape[0], dim), torch.float32, t.device)
    call("cesm_sinusoidal", P(t), P(emb), t.shape[0], dim, S())
    return emb


def linear_small(x, w, b, silu_in):
    R, I = x.shape
    O = w.shape[0]
    y = empty((R, O), torch.float32, x.device)
    call("cesm_linear_small_fwd", P(x), P(w), P(b), P(y), R, I, O, int(silu_in), S())
    return y


def linear_small_bwd(x, w, dy, dx, dw, db, silu_in, accumulate_dx):
    R, I = x.shape
    O = w.shape[0]
    call("cesm_linear_small_bwd", P(x), P(w), P(dy), P(dx), P(dw), P(db), R, I, O, int(silu_in), int(accumulate_dx),
         1, S())


def q_sample(x0, noise, t, sa, s1a):
    B = x0.shape[0]
    xt = empty(x0.shape, torch.float32, x0.device)
    call("cesm_q_sample", P(x0), P(noise), P(t), P(sa), P(s1a), P(xt), B, x0.numel() // B, S())
    return xt


def ddpm_step(x, eps, z, t, sra, betas, s1a, pv, out=None):
    """Fused DDPM ancestral update (model.py:168-183); z=None drops the noise term; out may be x."""
    B = x.shape[0]
    _chk(x, dtype=torch.float32)
    _chk(eps, x.shape, torch.float32)
    if z is not None:
        _chk(z, x.shape, torch.float32)
    if out is None:
        out = empty(x.shape, torch.float32, x.device)
    call("cesm_ddpm_step", P(x), P(eps), P(z), P(t), P(sra), P(betas), P(s1a), P(pv), P(out), B, x.numel() // B, S())
    return out


def mse(pred, tgt):
    loss = empty((), torch.float32, pred.device)
    part = empty((512,), torch.float32, pred.device)
    call("cesm_mse", P(pred), P(tgt), P(loss), P(part), pred.numel(), S())
    return loss


def mse_bwd(pred, tgt, gscale):
    d = empty(pred.shape, torch.float32, pred.device)
    call("cesm_mse_bwd", P(pred), P(tgt), P(gscale), P(d), pred.numel(), S())
    return d


def grad_norm(flat_grad, max_norm, loss=None):
    info = empty((4,), torch.float32, flat_grad.device)
    part = empty((1024,), torch.float64, flat_grad.device)
    call("cesm_grad_norm", P(flat_grad), flat_grad.numel(), float(max_norm), P(loss), P(part), P(info), S())
    return info


def adamw(p, g, m, v, info, lr, b1, b2, eps, wd, step_dev, use_clip):
    """step_dev: device int32 [1] step counter (advanced on device when the step is finite)"""
    _chk(step_dev, (1,), torch.int32)
    call("cesm_adamw", P(p), P(g), P(m), P(v), P(info), P(step_dev), p.numel(), float(lr), float(b1), float(b2),
         float(eps), float(wd), int(use_clip), S())


def cast(x, dtype):
    y = empty(x.shape, dtype, x.device)
    call("cesm_cast", dtcode(x), _DT[dtype], P(x), P(y), x.numel(), S())
    return y


def window_gather(cond, tgt, items, K, h, w, center):
    T, M, H, W = cond.shape
    n = items.shape[0]
    cwin = empty((n, 1, K, h, w), torch.float32, items.device)
    x0 = empty((n, 1, h, w), torch.float32, items.device)
    call("cesm_window_gather", P(cond), P(tgt), P(items), P(cwin), P(x0), n, K, M, H, W, h, w, int(center), S())
    return cwin, x0


def conv_fwd_variant(dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P, U):
    """name of the kernel cesm_conv_fwd selects for these arguments (host-only query)"""
    return lib().cesm_conv_fwd_variant(_DT[dtype], Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P, U).decode()


def tflash_bwd_variant(F, HW):
    """name of the dq kernel cesm_tflash_bwd selects (host-only query)"""
    return lib().cesm_tflash_bwd_variant(F, HW).decode()


def conv_wgrad_variant(dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P, U, with_bias=False):
    """name of the kernel cesm_conv_wgrad selects (host-only query)"""
    return lib().cesm_conv_wgrad_variant(_DT[dtype], Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P, U,
                                         int(bool(with_bias))).decode()
