"""UNetModel3D on libcesm_hip.so — the MI355X-native replacement for the reference's video_net.py.

The module tree (attribute names, parameter shapes, construction order) mirrors the reference
(video_net.py:562-764) so `state_dict()` keys are identical and a fixed torch seed yields the
reference's initial weights.  The `nn.Conv3d` / `nn.Linear` / `nn.GroupNorm` / `nn.Embedding`
children are parameter holders only: the forward and backward of the whole network run as an
explicit executor over HIP kernels on channels-last activations [B*F, H, W, C] (bf16 or fp32),
with the backward written out by hand (gradient fan-ins fused into the producing kernels'
epilogues) and parameter gradients written straight into `param.grad`.

Autograd sees the network as ONE node (`_NetFunction`): loss.backward() calls
`UNetModel3D.backward_from`.
"""
from __future__ import annotations

import math
import os
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import kernels as K


# Bumped by every in-place parameter update made through raw pointers (FusedAdamW.step):
# packed-weight caches key on it, since such updates are invisible to torch's version counters.
_PARAM_EPOCH = [0]


def bump_param_epoch():
    _PARAM_EPOCH[0] += 1


# ============================================================================ run context
# Weight gradients off the critical path: the backward's dX chain stays on the current stream and every
# parameter-gradient GEMM (conv / 1x1 / qkv wgrads, bias column sums, stem wgrad) is enqueued on a second
# HIP stream ordered after the kernel that produced its inputs.  The wgrads are HBM-bound (the level-0 qkv
# wgrad streams 4.4 GB) while the dX kernels are MFMA/latency-bound, so the two co-run on the CUs.
# "0" (default): off, "attn": only the fused attention blocks' wgrads, "1": every wgrad.  Rounds 3-4 saw 5-8x slower
# steps with "1" whenever the host ran ahead of the GPU; the cause was the allocator's record_stream reuse rule (see
# _Side), fixed in round 5.
WGRAD_STREAM = os.environ.get("CESM_WGRAD_STREAM", "0")
_WSTREAMS = {}


def _wgrad_stream(device):
    s = _WSTREAMS.get(device)
    if s is None:
        s = _WSTREAMS[device] = torch.cuda.Stream(device=device)
    return s


class _Side:
    """Context: enqueue on the wgrad stream after everything already on the current stream.  The tensors read there
    are kept alive by the run context until rc.join() has made the current stream wait for the wgrad stream; freed
    after that, their memory can only be reused by work ordered after the wgrad kernels.

    (Round 5: these tensors used to be `record_stream`-ed on the wgrad stream instead.  The caching allocator then
    reuses such a block only once the recorded event has completed, which it checks when it allocates; with the host
    running steps ahead of the GPU (no per-step synchronize, as in bench.py) the events are still pending, so every
    step took fresh segments from hipMalloc -- 171-223 hipMalloc calls over 3-4 steps, ~10 ms each with the device
    busy: the 5-8x slower steps of rounds 3-4, profiles/r5_wgrad_stream_trace.txt.)"""

    def __init__(self, rc, tensors):
        self.rc, self.tensors = rc, tensors

    def __enter__(self):
        ws = self.rc.wstream
        if ws is None:
            return
        ws.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.stream(ws)
        self._ctx.__enter__()

    def __exit__(self, *exc):
        ws = self.rc.wstream
        if ws is None:
            return False
        self._ctx.__exit__(*exc)
        self.rc.keep.extend(t for t in self.tensors if t is not None)
        return False


_NOSIDE = SimpleNamespace(wstream=None)


class RunCtx:
    """Per-call state: compute dtype, batch geometry, shared tables, weight-pack cache."""

    def __init__(self, net, B, F, cdt, save):
        self.net, self.B, self.F, self.cdt, self.save = net, B, F, cdt, save
        self.dt = None      # grad of the time embedding (allocated in backward)
        self.dtable = None  # grad of the rel-pos embedding table
        self.wstream = None  # weight-gradient stream (set by the backward when WGRAD_STREAM)
        self.keep = []  # tensors the wgrad stream reads, alive until released by checkpoint() / join()
        self._mark = None  # (event on the wgrad stream, len(keep)) at the last checkpoint

    def packed(self, w, cout, cin, kh, kw, swap, flip):
        return self.net._packed(w, self.cdt, cout, cin, kh, kw, swap, flip)

    def side(self, *tensors, attn=False):
        return _Side(self if (attn or WGRAD_STREAM == "1") else _NOSIDE, tensors)

    def checkpoint(self):
        """a module boundary of the backward: release the tensors of the wgrad work enqueued before the PREVIOUS boundary,
        once the current stream has been ordered after that work (round 6, ADVICE r5: join() alone kept every per-layer
        dy / x the wgrad stream read until the end of the backward).  One level of overlap stays; the kept set is
        bounded by about two levels' tensors."""
        if self.wstream is None:
            return
        ev = torch.cuda.Event()
        ev.record(self.wstream)
        if self._mark is not None:
            prev, n = self._mark
            torch.cuda.current_stream().wait_event(prev)
            del self.keep[:n]
        self._mark = (ev, len(self.keep))

    def join(self):
        """current stream waits for every weight gradient enqueued so far; the tensors they read may go after that"""
        if self.wstream is not None:
            torch.cuda.current_stream().wait_stream(self.wstream)
        self.keep.clear()
        self._mark = None


def gbuf(p):
    """fp32 gradient destination for parameter p (kernels accumulate into it)."""
    if p is None or not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
    return p.grad


def _wflat(p):
    """gradient buffer of a 1x1 conv weight [O, I, 1, 1] viewed as [O, I] (or None)"""
    g = gbuf(p)
    return None if g is None else g.view(g.shape[0], g.shape[1])


def _gflat(p):
    """flat view of p's gradient buffer (LayerNorm gamma [1, C, 1, 1, 1] -> [C]) or None"""
    g = gbuf(p)
    return None if g is None else g.view(-1)


# ============================================================================ conv helpers
class ConvSpec:
    """Geometry of one conv-like layer in GEMM terms (see csrc/conv.hip)."""

    def __init__(self, mod):
        w = mod.weight
        self.mod = mod
        self.transposed = isinstance(mod, nn.ConvTranspose3d)
        if isinstance(mod, nn.Linear):
            self.cout, self.cin, self.k, self.stride, self.pad = w.shape[0], w.shape[1], 1, 1, 0
        elif self.transposed:
            self.cin, self.cout, self.k = w.shape[0], w.shape[1], w.shape[-1]
            self.stride, self.pad = mod.stride[-1], mod.padding[-1]
        else:
            self.cout, self.cin, self.k = w.shape[0], w.shape[1], w.shape[-1]
            self.stride, self.pad = mod.stride[-1], mod.padding[-1]

    def out_hw(self, H, W):
        k, s, p = self.k, self.stride, self.pad
        if self.transposed:
            return (H - 1) * s - 2 * p + k, (W - 1) * s - 2 * p + k
        return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1

    # forward GEMM: (S, P, U, swap, flip)
    def fwd_map(self):
        if self.transposed:
            return 1, self.k - 1 - self.pad, self.stride, 1, 1
        return self.stride, self.pad, 1, 0, 0


def conv_forward(rc, spec, x1, x2=None, res=None):
    k = spec.k
    St, Pd, U, swap, flip = spec.fwd_map()
    Nb, H, W, _ = x1.shape
    Ho, Wo = spec.out_hw(H, W)
    wp = rc.packed(spec.mod.weight, spec.cout, spec.cin, k, k, swap, flip)
    geom = (Ho, Wo, spec.cout, k, k, St, Pd, U)
    y = K.conv_fwd(x1, x2, wp, spec.mod.bias, geom, res=res)
    st = SimpleNamespace(x1=x1, x2=x2, geom=geom, swap=swap, flip=flip) if rc.save else None
    return y, st


def conv_param_grads(spec, st, dy, dw, db):
    """dW (+ dbias) of one conv (called on the weight-gradient stream).  The bias gradient rides on the
    weight-gradient pass when its kernel supports it (bf16 wide-tile wgrad), else a column sum of dY."""
    if dw is not None:
        if spec.transposed:
            # the transposed conv's weight gradient sum_{a,b} x[a,b] (x) dOut[S*a - P + ky, S*b - P + kx] is the
            # weight gradient of the plain strided conv dOut -> x-grid (GEMM co = x channels = torch dim 0,
            # taps unflipped: lands in the [in, out, 1, k, k] layout with swap = flip = 0); every tap is live,
            # unlike the U = S gather form where 3/4 of the (pixel, tap) pairs are zero
            assert st.x2 is None
            Hx, Wx = st.x1.shape[1], st.x1.shape[2]
            K.conv_wgrad(dy, None, st.x1, None, dw, (Hx, Wx, spec.cin, spec.k, spec.k, spec.stride, spec.pad, 1), 0, 0)
        else:
            if K.conv_wgrad(st.x1, st.x2, dy, None, dw, st.geom, st.swap, st.flip, db=db):
                db = None
    if db is not None:
        K.colsum(dy, db)


def conv_backward(rc, spec, st, dy, need_dx=True, dres1=None, dres2=None, bias_done=False):
    """Param grads of the conv + (optionally) dX (split for concat inputs) + fused residual grads.
    bias_done: the bias gradient was already produced (by the GroupNorm backward's reduction)."""
    w, b = spec.mod.weight, spec.mod.bias
    dw = gbuf(w)
    db = gbuf(b)
    with rc.side(dy, st.x1, st.x2):
        conv_param_grads(spec, st, dy, dw, None if bias_done else db)
    if not need_dx:
        return None
    k = spec.k
    Nb, H, W, C1 = st.x1.shape
    cin = spec.cin
    if spec.transposed:
        # dIn = plain strided conv of dOut; GEMM co = Cin_t (torch dim 0)
        wp = rc.packed(w, cin, spec.cout, k, k, 0, 0)
        geom = (H, W, cin, k, k, spec.stride, spec.pad, 1)
    else:
        # dX = transposed conv of dY (stride 1: flipped conv); GEMM co = Cin (torch dim 1)
        wp = rc.packed(w, cin, spec.cout, k, k, 1, 1)
        geom = (H, W, cin, k, k, 1, k - 1 - spec.pad, spec.stride)
    split = C1 if st.x2 is not None else None
    return K.conv_fwd(dy, None, wp, None, geom, res=dres1, res2=dres2, out_split=split)


# the fused to_qkv backward only at C = 64 (the decadal window's level 0: 3.49 vs 3.75 ms per call); at C >= 128 every
# 64-channel slice re-reads dqkv and the dgrad GEMM + wide weight-gradient pair is faster (0.84-0.95x,
# profiles/r6c_qkv_time.txt)
QKV_BWD_MAXC = 64


def qkv_backward(rc, spec, st, dqkv):
    """backward of a to_qkv projection (768 outputs, no bias) on the unfused attention paths: dn and (+=) its weight
    gradient, with dqkv read once by the fused kernel (csrc/qkvbwd.hip, round 6) in bf16; otherwise the dgrad GEMM +
    weight-gradient GEMM of conv_backward."""
    n = st.x1
    Nb, H, W, C = n.shape
    if (n.dtype == torch.bfloat16 and C == QKV_BWD_MAXC and st.x2 is None and spec.k == 1 and spec.cout == 768
            and spec.mod.bias is None and not spec.transposed and K.qkv_bwd_supported(Nb * H * W, C)):
        wt = rc.packed(spec.mod.weight, C, 768, 1, 1, 1, 1)
        dw = gbuf(spec.mod.weight)
        return K.qkv_bwd(dqkv, n, wt, None if dw is None else dw.view(768, C))
    return conv_backward(rc, spec, st, dqkv)


# ============================================================================ modules
class Residual(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn


class LayerNorm(nn.Module):
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(1, dim, 1, 1, 1))


class PreNorm(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.fn = fn
        self.norm = LayerNorm(dim)


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class RotaryEmbedding(nn.Module):
    """rotary_embedding.py:62-134 — only the frozen `freqs` parameter is state."""

    def __init__(self, dim, theta=10000):
        super().__init__()
        freqs = 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))
        self.freqs = nn.Parameter(freqs, requires_grad=False)


class RelativePositionBias(nn.Module):
    def __init__(self, heads=8, num_buckets=32, max_distance=128):
        super().__init__()
        self.num_buckets = num_buckets
        self.max_distance = max_distance
        self.relative_attention_bias = nn.Embedding(num_buckets, heads)


class EinopsToAndFrom(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn


class Attention(nn.Module):
    def __init__(self, dim, heads=8, dim_head=32, rotary_emb=None):
        super().__init__()
        assert heads == 8 and dim_head == 32, "kernels are specialised for 8 heads x 32"
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.rotary_emb = rotary_emb
        self.to_qkv = nn.Linear(dim, dim_head * heads * 3, bias=False)
        self.to_out = nn.Linear(dim_head * heads, dim, bias=False)


class SpatialLinearAttention(nn.Module):
    def __init__(self, dim, heads=8, dim_head=32):
        super().__init__()
        assert heads == 8 and dim_head == 32, "kernels are specialised for 8 heads x 32"
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.to_qkv = nn.Conv2d(dim, dim_head * heads * 3, 1, bias=False)
        self.to_out = nn.Conv2d(dim_head * heads, dim, 1)


class Block(nn.Module):
    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.proj = nn.Conv3d(dim, dim_out, (1, 3, 3), padding=(0, 1, 1))
        self.norm = nn.GroupNorm(groups, dim_out)


class ResnetBlock(nn.Module):
    def __init__(self, dim, dim_out, *, time_emb_dim=None, groups=8):
        super().__init__()
        self.mlp = (nn.Sequential(nn.SiLU(), nn.Linear(time_emb_dim, dim_out * 2))
                    if time_emb_dim is not None else None)
        self.block1 = Block(dim, dim_out, groups=groups)
        self.block2 = Block(dim_out, dim_out, groups=groups)
        self.res_conv = nn.Conv3d(dim, dim_out, 1) if dim != dim_out else nn.Identity()


def Downsample(dim):
    return nn.Conv3d(dim, dim, (1, 4, 4), (1, 2, 2), (0, 1, 1))


def Upsample(dim):
    return nn.ConvTranspose3d(dim, dim, (1, 4, 4), (1, 2, 2), (0, 1, 1))


# ============================================================================ layer executors
def _flat(p):
    return p.reshape(-1)


# GroupNorm statistics from partials written by the Block conv's epilogue (halo conv kernels) instead of a
# separate pass over y (round 2: the pass took 2.06 ms per step, the epilogue partials ~+3 % of the convs)
GN_EPI_STATS = True


def block_fwd(rc, blk, x1, x2, ss, res):
    """Block (video_net.py:212-227): conv3x3 -> GroupNorm -> scale/shift -> SiLU (+res)."""
    spec = ConvSpec(blk.proj)
    G = blk.norm.num_groups
    Nb, H, W, _ = x1.shape
    geom_hw = spec.out_hw(H, W)
    nslot = 0
    if GN_EPI_STATS and x1.dtype == torch.bfloat16 and spec.cout % (4 * G) == 0:
        St, Pd, U, swap, flip = spec.fwd_map()
        geom = (geom_hw[0], geom_hw[1], spec.cout, spec.k, spec.k, St, Pd, U)
        nslot = K.conv_gn_nslot(x1, x2, geom, rc.B)
    if nslot > 0:
        wp = rc.packed(spec.mod.weight, spec.cout, spec.cin, spec.k, spec.k, swap, flip)
        y, part = K.conv_fwd_gn(x1, x2, wp, spec.mod.bias, geom, rc.B, nslot)
        cst = SimpleNamespace(x1=x1, x2=x2, geom=geom, swap=swap, flip=flip) if rc.save else None
        stats = K.gn_stats_part(part, y.numel() // (spec.cout * rc.B), G, blk.norm.eps)
    else:
        y, cst = conv_forward(rc, spec, x1, x2)
        stats = K.gn_stats(y, rc.B, G, blk.norm.eps)
    out = K.gn_apply(y, stats, blk.norm.weight, blk.norm.bias, ss, res, rc.B, G)
    st = SimpleNamespace(spec=spec, cst=cst, y=y, stats=stats, ss=ss) if rc.save else None
    return out, st


def block_bwd(rc, blk, st, dout, want_dss, dres1=None, dres2=None):
    G = blk.norm.num_groups
    dy, dss = K.gn_bwd(dout, st.y, st.stats, blk.norm.weight, blk.norm.bias, st.ss, gbuf(blk.norm.weight),
                       gbuf(blk.norm.bias), rc.B, G, want_dss, dbias=gbuf(blk.proj.bias))
    dx = conv_backward(rc, st.spec, st.cst, dy, True, dres1, dres2, bias_done=True)
    return dx, dss


def resnet_fwd(rc, rb, x1, x2=None, temb=None):
    """ResnetBlock (video_net.py:230-265)."""
    ss = None
    if rb.mlp is not None:
        lin = rb.mlp[1]
        ss = K.linear_small(temb, lin.weight, lin.bias, True)  # SiLU -> Linear, [B, 2*dout]
    h, st1 = block_fwd(rc, rb.block1, x1, x2, ss, None)
    rst = None
    if isinstance(rb.res_conv, nn.Identity):
        r = x1
    else:
        rspec = ConvSpec(rb.res_conv)
        r, rst = conv_forward(rc, rspec, x1, x2)
    out, st2 = block_fwd(rc, rb.block2, h, None, None, r)
    st = SimpleNamespace(st1=st1, st2=st2, rst=rst, temb=temb) if rc.save else None
    return out, st


def resnet_bwd(rc, rb, st, dout):
    dh, _ = block_bwd(rc, rb.block2, st.st2, dout, False)
    if isinstance(rb.res_conv, nn.Identity):
        dr = (dout, None)
    else:
        r = conv_backward(rc, ConvSpec(rb.res_conv), st.rst, dout, True)
        dr = r if isinstance(r, tuple) else (r, None)
    dx, dss = block_bwd(rc, rb.block1, st.st1, dh, rb.mlp is not None, dr[0], dr[1])
    if rb.mlp is not None:
        lin = rb.mlp[1]
        K.linear_small_bwd(st.temb, lin.weight, dss, rc.dt, gbuf(lin.weight), gbuf(lin.bias), True, True)
    return dx  # tensor, or (dx1, dx2) for concat inputs


# widest channel count routed to the fused kernels: below it the 768-channel qkv intermediate is what
# costs (HBM); above it the level is small and the unfused GEMMs are cheaper than per-pixel-group
# weight re-reads (C = 256 / 512: unfused measured faster, rounds 1-2)
FUSED_TBLOCK_MAXC = 128
# widest C whose fused temporal forward writes O for the to_out weight gradient; above it the fused backward emits O
# (round 6 A/B at C = 128: profiles/r6i_*)
TBLOCK_FWD_O_MAXC = 256


def _tblock_fused(rc, C):
    return rc.cdt == torch.bfloat16 and rc.F <= 16 and C in K.TBLOCK_C and C <= FUSED_TBLOCK_MAXC


# head-parallel backward with in-kernel weight gradients (C = 64, F <= 12): no 768-channel dqkv round trip.  The
# backward recomputes O = P V from its own P and writes it for a wide to_out weight-gradient GEMM with dy (round 6: the
# forward's O write cost 477 us of a 1892 us level-0 call, tools/fwd_o_cost.py; the in-kernel to_out gradient measured
# slower, round 5: 32 more accumulators took twh_bwd from 9 to 58-93 spilled registers and 3.3 to 5.3 ms per call).
def _tblock_dw(rc, x):
    Nb, H, W, C = x.shape
    return _tblock_fused(rc, C) and K.tblock_bwd_dw_supported(rc.B, rc.F, H * W, C)


# pixel-major qkv for the long-window attention core (round 4: a pixel's frames as adjacent rows, F = 120 step
# 234.4-235.1 -> 232.0-232.3 ms)
def _tf_pixel_major(rc, x):
    return rc.F > 16 and x.dtype == torch.bfloat16 and K.lib().cesm_tflash_supported(rc.F) == 1


def tattn_fwd(rc, res_mod, x):
    """Residual(PreNorm(EinopsToAndFrom(Attention))) over frames (video_net.py:368-454).
    bf16: one fused kernel (csrc/tblock.hip); fp32 parity mode: LN -> to_qkv -> core -> to_out."""
    pre = res_mod.fn
    attn = pre.fn.fn
    Nb, H, W, C = x.shape
    HW = H * W
    if rc.F == 1 and not rc.save:
        # single frame (the sampler's F = 1 forward, inference.py:229): softmax over one key is exactly 1,
        # so the block is x + to_out(v) — q, k, RoPE and the rel-pos bias drop out.
        # LN -> v rows of to_qkv (1x1 GEMM) -> to_out with the residual fused.
        n, _ = K.ln_fwd(x, _flat(pre.norm.gamma), save=False, eps=pre.norm.eps)
        wv = rc.packed(attn.to_qkv.weight[512:768], 256, C, 1, 1, 0, 0)
        v = K.conv_fwd(n, None, wv, None, (H, W, 256, 1, 1, 1, 0, 1))
        wo = rc.packed(attn.to_out.weight, C, 256, 1, 1, 0, 0)
        return K.conv_fwd(v, None, wo, None, (H, W, C, 1, 1, 1, 0, 1), res=x), None
    if _tblock_dw(rc, x):
        # gamma folded into the QKV weights (images built from the fp32 master weight); the backward computes
        # the to_qkv and gamma gradients in-kernel, and O for the to_out gradient.
        wo = rc.packed(attn.to_out.weight, C, 256, 1, 1, 0, 0)
        y, mr, lse, _ = K.tblock_fwd_fold(x, _flat(pre.norm.gamma), attn.to_qkv.weight, wo, rc.bias, rc.rot, rc.B,
                                          rc.F, attn.scale, save=rc.save, eps=pre.norm.eps, save_o=False)
        st = SimpleNamespace(fused=True, fold=True, x=x, mr=mr, lse=lse) if rc.save else None
        return y, st
    if _tblock_fused(rc, C):
        wq = rc.packed(attn.to_qkv.weight, 768, C, 1, 1, 0, 0)
        wo = rc.packed(attn.to_out.weight, C, 256, 1, 1, 0, 0)
        # training: the forward also writes O (to_out's input) so the backward does not emit it
        save_o = rc.save and C <= TBLOCK_FWD_O_MAXC
        y, mr, lse, o = K.tblock_fwd(x, _flat(pre.norm.gamma), wq, wo, rc.bias, rc.rot, rc.B, rc.F, attn.scale,
                                     save=rc.save, eps=pre.norm.eps, save_o=save_o)
        st = SimpleNamespace(fused=True, fold=False, x=x, mr=mr, lse=lse, o=o) if rc.save else None
        return y, st
    # long windows (MFMA core, F > 16): the LN output -- and with it the to_qkv GEMM's qkv rows and, in the backward,
    # dqkv and dn -- in pixel-major order, so the attention kernels read a pixel's frames as adjacent rows
    pm = _tf_pixel_major(rc, x)
    perm = (rc.F, HW) if pm else None
    n, mr = K.ln_fwd(x, _flat(pre.norm.gamma), save=rc.save, eps=pre.norm.eps, perm=perm)
    qspec, ospec = ConvSpec(attn.to_qkv), ConvSpec(attn.to_out)
    qkv, qst = conv_forward(rc, qspec, n)
    o, lse = K.tattn_fwd(qkv.view(-1, 768), rc.bias, rc.rot, rc.B, rc.F, HW, attn.scale, save=rc.save,
                         pixel_major=pm)
    y, ost = conv_forward(rc, ospec, o.view(Nb, H, W, 256), None, res=x)
    st = SimpleNamespace(fused=False, x=x, mr=mr, qkv=qkv, o=o, lse=lse, qst=qst, ost=ost, perm=perm) if rc.save else None
    return y, st


def tattn_bwd(rc, res_mod, st, dy):
    pre = res_mod.fn
    attn = pre.fn.fn
    Nb, H, W, C = st.x.shape
    if st.fused and st.fold:
        wo_t = rc.packed(attn.to_out.weight, 256, C, 1, 1, 1, 1)
        dwo = gbuf(attn.to_out.weight)
        r = K.tblock_bwd_dw(st.x, dy, st.mr, st.lse, attn.to_qkv.weight, _flat(pre.norm.gamma), wo_t, rc.bias, rc.rot,
                            gbuf(attn.to_qkv.weight), _gflat(pre.norm.gamma), rc.dtable, rc.B, rc.F, attn.scale,
                            emit_o=dwo is not None)
        if dwo is None:
            return r
        dx, o = r
        with rc.side(o, dy, attn=True):
            K.conv_wgrad(o, None, dy, None, dwo, (H, W, C, 1, 1, 1, 0, 1), 0, 0)
        return dx
    if st.fused:
        wq = rc.packed(attn.to_qkv.weight, 768, C, 1, 1, 0, 0)
        wq_t = rc.packed(attn.to_qkv.weight, C, 768, 1, 1, 1, 1)
        wo_t = rc.packed(attn.to_out.weight, 256, C, 1, 1, 1, 1)
        dwq, dwo = gbuf(attn.to_qkv.weight), gbuf(attn.to_out.weight)
        want = dwq is not None or dwo is not None
        dx, dqkv, o, xn = K.tblock_bwd(st.x, dy, _flat(pre.norm.gamma), st.mr, st.lse, wq, wq_t, wo_t, rc.bias,
                                       rc.rot, gbuf(pre.norm.gamma), rc.dtable, rc.B, rc.F, attn.scale,
                                       want_wgrad_inputs=want, emit_o=st.o is None)
        if st.o is not None:
            o = st.o
        with rc.side(xn, dqkv, o, dy, attn=True):
            if dwq is not None:
                K.conv_wgrad(xn, None, dqkv, None, dwq, (H, W, 768, 1, 1, 1, 0, 1), 0, 0)
            if dwo is not None:
                K.conv_wgrad(o, None, dy, None, dwo, (H, W, C, 1, 1, 1, 0, 1), 0, 0)
        return dx
    do = conv_backward(rc, ConvSpec(attn.to_out), st.ost, dy)
    dqkv = K.tattn_bwd(st.qkv.view(-1, 768), st.o, do.view(-1, 256), st.lse, rc.bias, rc.rot, rc.dtable, rc.B,
                       rc.F, H * W, attn.scale, pixel_major=st.perm is not None)
    dn = qkv_backward(rc, ConvSpec(attn.to_qkv), st.qst, dqkv.view(Nb, H, W, 768))
    return K.ln_bwd(dn, st.x, st.mr, _flat(pre.norm.gamma), gbuf(pre.norm.gamma), dres=dy, perm=st.perm)


def _sla_fused(rc, C):
    return rc.cdt == torch.bfloat16 and C in K.SLAF_C


_ONES = {}


def _ones(C, device):
    t = _ONES.get((C, device))
    if t is None:
        t = _ONES[(C, device)] = torch.ones(C, device=device)
    return t


# head-parallel SLA backward with in-kernel weight gradients (C = 64), the to_out weight / bias gradients from the
# recomputed q~ and the forward's context (no 256-channel O written by the forward; round 2: 58.44 -> 59.30 samples/s)
def _sla_dw(rc, x):
    Nb, H, W, C = x.shape
    return _sla_fused(rc, C) and K.slaf_bwd_dw_supported(Nb, H * W, C)


def sla_fwd(rc, res_mod, x):
    """Residual(PreNorm(SpatialLinearAttention)) per frame (video_net.py:313-347).
    bf16, C=64: fused kernels (csrc/sla_fused.hip); otherwise LN -> to_qkv -> core -> to_out."""
    pre = res_mod.fn
    sla = pre.fn
    Nb, H, W, C = x.shape
    if _sla_dw(rc, x):
        # LN gamma folded into the QKV weights (unit gamma in the kernels): the backward then produces the
        # to_qkv and gamma gradients in-kernel, and the to_out gradients from the recomputed q~ and the saved
        # context, so O is not written.
        gamma = _flat(pre.norm.gamma)
        wq_fold = K.pack_scaled(sla.to_qkv.weight.reshape(768, C), gamma)
        wo = rc.packed(sla.to_out.weight, C, 256, 1, 1, 0, 0)
        ones = _ones(C, x.device)
        y, state = K.slaf_fwd(x, ones, wq_fold, wo, sla.to_out.bias, sla.scale, eps=pre.norm.eps, save_o=False)
        st = SimpleNamespace(fused=True, fold=True, x=x, state=state, wq_fold=wq_fold) if rc.save else None
        return y, st
    if _sla_fused(rc, C):
        wq = rc.packed(sla.to_qkv.weight, 768, C, 1, 1, 0, 0)
        wo = rc.packed(sla.to_out.weight, C, 256, 1, 1, 0, 0)
        # training: the forward also writes O (to_out's input) so the backward does not emit it
        y, state = K.slaf_fwd(x, _flat(pre.norm.gamma), wq, wo, sla.to_out.bias, sla.scale, eps=pre.norm.eps,
                              save_o=rc.save)
        st = SimpleNamespace(fused=True, fold=False, x=x, state=state) if rc.save else None
        return y, st
    n, mr = K.ln_fwd(x, _flat(pre.norm.gamma), save=rc.save, eps=pre.norm.eps)
    qkv, qst = conv_forward(rc, ConvSpec(sla.to_qkv), n)
    o, ctx, ml = K.sla_fwd(qkv.view(-1, 768), Nb, H * W, sla.scale)
    y, ost = conv_forward(rc, ConvSpec(sla.to_out), o.view(Nb, H, W, 256), None, res=x)
    st = SimpleNamespace(fused=False, x=x, mr=mr, qkv=qkv, ctx=ctx, ml=ml, qst=qst, ost=ost) if rc.save else None
    return y, st


def sla_bwd(rc, res_mod, st, dy):
    pre = res_mod.fn
    sla = pre.fn
    Nb, H, W, C = st.x.shape
    if st.fused and st.fold:
        wo_t = rc.packed(sla.to_out.weight, 256, C, 1, 1, 1, 1)
        dwo, dbo = gbuf(sla.to_out.weight), gbuf(sla.to_out.bias)
        if (dwo is None) != (dbo is None):  # one of the two frozen: a scratch destination
            dwo = dwo if dwo is not None else torch.zeros_like(sla.to_out.weight)
            dbo = dbo if dbo is not None else torch.zeros_like(sla.to_out.bias)
        # to_out gradients from the dctx pass (the forward wrote no O)
        return K.slaf_bwd_dw(st.x, dy, _ones(C, dy.device), st.wq_fold, sla.to_qkv.weight.reshape(768, C),
                             _flat(pre.norm.gamma), wo_t, st.state, _wflat(sla.to_qkv.weight), _gflat(pre.norm.gamma),
                             sla.scale, eps=pre.norm.eps, dwout=dwo.view(C, 256) if dwo is not None else None,
                             dbout=dbo if dwo is not None else None)
    if st.fused:
        wq = rc.packed(sla.to_qkv.weight, 768, C, 1, 1, 0, 0)
        wq_t = rc.packed(sla.to_qkv.weight, C, 768, 1, 1, 1, 1)
        wo_t = rc.packed(sla.to_out.weight, 256, C, 1, 1, 1, 1)
        dwq, dwo, dbo = gbuf(sla.to_qkv.weight), gbuf(sla.to_out.weight), gbuf(sla.to_out.bias)
        dx, dqkv, o, xn = K.slaf_bwd(st.x, dy, _flat(pre.norm.gamma), wq, wq_t, wo_t, st.state,
                                     gbuf(pre.norm.gamma), sla.scale,
                                     want_wgrad_inputs=dwq is not None or dwo is not None, eps=pre.norm.eps)
        with rc.side(xn, dqkv, o, dy, attn=True):
            if dwq is not None:
                K.conv_wgrad(xn, None, dqkv, None, dwq, (H, W, 768, 1, 1, 1, 0, 1), 0, 0)
            if dwo is not None and K.conv_wgrad(o, None, dy, None, dwo, (H, W, C, 1, 1, 1, 0, 1), 0, 0, db=dbo):
                dbo = None
            if dbo is not None:
                K.colsum(dy, dbo)
        return dx
    do = conv_backward(rc, ConvSpec(sla.to_out), st.ost, dy)
    dqkv = K.sla_bwd(st.qkv.view(-1, 768), do.view(-1, 256), st.ctx, st.ml, Nb, H * W, sla.scale)
    dn = qkv_backward(rc, ConvSpec(sla.to_qkv), st.qst, dqkv.view(Nb, H, W, 768))
    return K.ln_bwd(dn, st.x, st.mr, _flat(pre.norm.gamma), gbuf(pre.norm.gamma), dres=dy)


# ============================================================================ the network
class UNetModel3D(nn.Module):
    def __init__(self, n_vars, model_dim, dim_mults=(1, 2, 4, 8), attn_heads=8, attn_dim_head=32,
                 use_sparse_linear_attn=True, use_mid_attn=False, init_kernel_size=7, resnet_groups=8,
                 use_checkpoint=False, use_temp_attn=True, day_cond=False, year_cond=False, cond_map=True):
        super().__init__()
        if not (use_temp_attn and cond_map) or day_cond or year_cond or use_mid_attn:
            raise NotImplementedError("only the configuration model.UNet builds is supported "
                                      "(temporal attention, cond map, no day/year cond, no mid attn)")
        if n_vars != 1:
            raise NotImplementedError("n_vars must be 1 (single target variable)")
        self.compute_dtype = torch.bfloat16
        in_ch = 2 * n_vars
        pad = init_kernel_size // 2
        self.input_conv = nn.Conv3d(in_ch, model_dim, (1, init_kernel_size, init_kernel_size),
                                    padding=(0, pad, pad))
        rotary = RotaryEmbedding(min(32, attn_dim_head))
        self.time_rel_pos_bias = RelativePositionBias(heads=attn_heads, max_distance=32)
        self.time_rel_pos_bias = RelativePositionBias(heads=attn_heads, max_distance=32)

        def tattn(dim):
            return EinopsToAndFrom(Attention(dim, heads=attn_heads, dim_head=attn_dim_head, rotary_emb=rotary))

        self.input_temp_op = Residual(PreNorm(model_dim, tattn(model_dim)))
        dims = [model_dim, *[int(model_dim * m) for m in dim_mults]]
        in_out = list(zip(dims[:-1], dims[1:]))
        time_dim = model_dim * 4
        self.time_mlp = nn.Sequential(SinusoidalPosEmb(model_dim), nn.Linear(model_dim, time_dim), nn.SiLU(),
                                      nn.Linear(time_dim, time_dim))
        self.downs = nn.ModuleList([])
        self.ups = nn.ModuleList([])
        nres = len(in_out)

        def rb(a, b):
            return ResnetBlock(a, b, time_emb_dim=time_dim, groups=resnet_groups)

        def sla(d):
            return Residual(PreNorm(d, SpatialLinearAttention(d, heads=attn_heads)))

        for i, (din, dout) in enumerate(in_out):
            last = i >= nres - 1
            self.downs.append(nn.ModuleList([
                rb(din, dout), rb(dout, dout),
                sla(dout) if use_sparse_linear_attn else nn.Identity(),
                Residual(PreNorm(dout, tattn(dout))),
                Downsample(dout) if not last else nn.Identity(),
            ]))
        mid = dims[-1]
        self.mid_block1 = rb(mid, mid)
        self.mid_spatial_attn = nn.Identity()
        self.mid_temporal_attn = Residual(PreNorm(mid, tattn(mid)))
        self.mid_block2 = rb(mid, mid)
        for i, (din, dout) in enumerate(reversed(in_out)):
            last = i >= nres - 1
            self.ups.append(nn.ModuleList([
                rb(dout * 2, din), rb(din, din),
                sla(din) if use_sparse_linear_attn else nn.Identity(),
                Residual(PreNorm(din, tattn(din))),
                Upsample(din) if not last else nn.Identity(),
            ]))
        self.out_conv = nn.Sequential(ResnetBlock(model_dim * 2, model_dim, groups=resnet_groups),
                                      nn.Conv3d(model_dim, n_vars, 1))
        self._pack_cache = {}
        self._pack_tables = {}  # dtype -> device int64 job table of the cached packs
        self._weights_epoch = 0

    # ---------------------------------------------------------------- weight packing cache
    def invalidate_packed(self):
        """Called after any in-place parameter update made through raw pointers (optimizer)."""
        self._weights_epoch += 1
        self._pack_cache.clear()
        self._pack_tables.clear()

    def _packed(self, w, cdt, cout, cin, kh, kw, swap, flip):
        """GEMM-layout copy of conv weight w (cesm_conv_pack).  Packs persist across steps: after an
        optimizer step (epoch change) the first request re-packs EVERY cached weight in one batched
        launch (cesm_conv_pack_batch) instead of ~180 small ones."""
        key = (w.data_ptr(), cdt, cout, cin, kh, kw, swap, flip)
        ep = (self._weights_epoch, _PARAM_EPOCH[0])
        e = self._pack_cache.get(key)
        if e is not None and e.epoch == ep and e.version == w._version:
            return e.out
        if e is None:
            out = K.conv_pack(w.detach().reshape(w.shape), cdt, cout, cin, kh, kw, swap, flip)
            self._pack_cache[key] = SimpleNamespace(w=w, out=out, geo=(cout, cin, kh, kw, swap, flip), epoch=ep,
                                                    version=w._version)
            self._pack_tables.clear()
            return out
        if e.epoch != ep:
            self._repack_all(ep)
        if e.version != w._version:  # in-place update through torch (version counter), this weight only
            K.conv_pack_into(w.detach(), e.out, *e.geo)
            e.version = w._version
        e.epoch = ep
        return e.out

    def _repack_all(self, ep):
        for cdt in (torch.bfloat16, torch.float32):
            ents = [e for e in self._pack_cache.values() if e.out.dtype == cdt]
            if not ents:
                continue
            tab = self._pack_tables.get(cdt)
            if tab is None:
                assert all(e.out.numel() < 2 ** 31 for e in ents)  # the batch kernel indexes in 32 bits
                rows = [[e.w.data_ptr(), e.out.data_ptr(), *e.geo] for e in ents]
                tab = self._pack_tables[cdt] = K.conv_pack_table(rows, ents[0].out.device)
            K.conv_pack_batch(tab[0], len(ents), cdt, tab[1])
            for e in ents:
                e.epoch, e.version = ep, e.w._version

    # ---------------------------------------------------------------- executor
    def run_forward(self, x_t, cond, t, save):
        """x_t [B,Fx,H,W], cond [B,Fc,H,W] fp32 (frame axis already squeezed), t int64 [B]."""
        B, Fx, H, W = x_t.shape
        F = max(Fx, cond.shape[1])
        cdt = self.compute_dtype
        rc = RunCtx(self, B, F, cdt, save)
        rpb = self.time_rel_pos_bias
        rc.bias = K.relpos_fwd(rpb.relative_attention_bias.weight, F, rpb.num_buckets, rpb.max_distance)
        rc.rot = K.rope_table(self.input_temp_op.fn.fn.fn.rotary_emb.freqs, F)
        tape = SimpleNamespace(rc=rc, x_t=x_t, cond=cond, downs=[], ups=[])

        x = K.stem_fwd(x_t, cond, self.input_conv.weight, self.input_conv.bias, F, cdt)
        tape.stem_out = x
        x, tape.in_attn = tattn_fwd(rc, self.input_temp_op, x)
        r = x
        emb = K.sinusoidal(t, self.time_mlp[0].dim)
        h1 = K.linear_small(emb, self.time_mlp[1].weight, self.time_mlp[1].bias, False)
        temb = K.linear_small(h1, self.time_mlp[3].weight, self.time_mlp[3].bias, True)
        tape.emb, tape.h1 = emb, h1
        hs = []
        for b1, b2, sa, ta, down in self.downs:
            s = SimpleNamespace()
            x, s.b1 = resnet_fwd(rc, b1, x, None, temb)
            x, s.b2 = resnet_fwd(rc, b2, x, None, temb)
            if not isinstance(sa, nn.Identity):
                x, s.sa = sla_fwd(rc, sa, x)
            x, s.ta = tattn_fwd(rc, ta, x)
            hs.append(x)
            s.down = None
            if not isinstance(down, nn.Identity):
                x, s.down = conv_forward(rc, ConvSpec(down), x)
            tape.downs.append(s)
        x, tape.mid1 = resnet_fwd(rc, self.mid_block1, x, None, temb)
        x, tape.mid_attn = tattn_fwd(rc, self.mid_temporal_attn, x)
        x, tape.mid2 = resnet_fwd(rc, self.mid_block2, x, None, temb)
        for b1, b2, sa, ta, up in self.ups:
            s = SimpleNamespace()
            skip = hs.pop()
            x, s.b1 = resnet_fwd(rc, b1, x, skip, temb)
            x, s.b2 = resnet_fwd(rc, b2, x, None, temb)
            if not isinstance(sa, nn.Identity):
                x, s.sa = sla_fwd(rc, sa, x)
            x, s.ta = tattn_fwd(rc, ta, x)
            s.up = None
            if not isinstance(up, nn.Identity):
                x, s.up = conv_forward(rc, ConvSpec(up), x)
            tape.ups.append(s)
        x, tape.out_rb = resnet_fwd(rc, self.out_conv[0], x, r, None)
        head = self.out_conv[1]
        out = K.head_fwd(x, head.weight.reshape(-1), head.bias, B, F)
        tape.head_in = x
        return (out, tape) if save else out

    def backward_from(self, dout, tape):
        """backward of the forward that recorded `tape` (held by that forward's autograd node, so several
        grad-enabled forwards may be in flight and each backward replays its own activations)."""
        if tape is None:
            raise RuntimeError("backward called twice for one forward (its tape was already consumed)")
        rc = tape.rc
        dev = dout.device
        hook = getattr(self, "_grad_ready", None)

        def done(*mods):  # data-parallel overlap: these modules' gradients are final (distributed.arm)
            if hook is not None:
                hook([p for m in mods for p in m.parameters()], rc.wstream)
            rc.checkpoint()
        if WGRAD_STREAM != "0" and dout.is_cuda:
            rc.wstream = _wgrad_stream(dev)
        rc.dt = torch.zeros((rc.B, self.time_mlp[1].out_features), dtype=torch.float32, device=dev)
        rc.dtable = gbuf(self.time_rel_pos_bias.relative_attention_bias.weight)
        head = self.out_conv[1]
        hw, hb = gbuf(head.weight), gbuf(head.bias)
        dx = K.head_bwd(dout.contiguous(), tape.head_in, head.weight.reshape(-1),
                        None if hw is None else hw.view(-1), hb, rc.B, rc.F)
        dx, dr = resnet_bwd(rc, self.out_conv[0], tape.out_rb, dx)
        done(self.out_conv)
        nres = len(self.downs)
        dskips = [None] * nres
        for j in reversed(range(len(self.ups))):
            b1, b2, sa, ta, up = self.ups[j]
            s = tape.ups[j]
            if s.up is not None:
                dx = conv_backward(rc, ConvSpec(up), s.up, dx)
            dx = tattn_bwd(rc, ta, s.ta, dx)
            if not isinstance(sa, nn.Identity):
                dx = sla_bwd(rc, sa, s.sa, dx)
            dx = resnet_bwd(rc, b2, s.b2, dx)
            dx, dskip = resnet_bwd(rc, b1, s.b1, dx)
            dskips[nres - 1 - j] = dskip
            done(self.ups[j])
        dx = resnet_bwd(rc, self.mid_block2, tape.mid2, dx)
        dx = tattn_bwd(rc, self.mid_temporal_attn, tape.mid_attn, dx)
        dx = resnet_bwd(rc, self.mid_block1, tape.mid1, dx)
        done(self.mid_block1, self.mid_temporal_attn, self.mid_block2)
        for i in reversed(range(nres)):
            b1, b2, sa, ta, down = self.downs[i]
            s = tape.downs[i]
            if s.down is not None:
                dx = conv_backward(rc, ConvSpec(down), s.down, dx, True, dres1=dskips[i])
            else:
                dx = K.add(dx, dskips[i])
            dx = tattn_bwd(rc, ta, s.ta, dx)
            if not isinstance(sa, nn.Identity):
                dx = sla_bwd(rc, sa, s.sa, dx)
            dx = resnet_bwd(rc, b2, s.b2, dx)
            dx = resnet_bwd(rc, b1, s.b1, dx)
            done(self.downs[i])
        dx = K.add(dx, dr)
        dx = tattn_bwd(rc, self.input_temp_op, tape.in_attn, dx)
        wi, bi = gbuf(self.input_conv.weight), gbuf(self.input_conv.bias)
        with rc.side(tape.x_t, tape.cond, dx):
            if wi is not None:
                K.stem_wgrad(tape.x_t, tape.cond, dx, wi, rc.F)
            if bi is not None:
                K.colsum(dx, bi)
        # time MLP: temb = Lin3(SiLU(Lin1(emb)))
        l1, l3 = self.time_mlp[1], self.time_mlp[3]
        dh1 = torch.empty_like(tape.h1)
        K.linear_small_bwd(tape.h1, l3.weight, rc.dt, dh1, gbuf(l3.weight), gbuf(l3.bias), True, False)
        K.linear_small_bwd(tape.emb, l1.weight, dh1, None, gbuf(l1.weight), gbuf(l1.bias), False, False)
        rc.join()


class _NetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net, x_t, cond, t, anchor):
        ctx.net = net
        out, ctx.tape = net.run_forward(x_t, cond, t, save=True)
        return out

    @staticmethod
    def backward(ctx, dout):
        tape, ctx.tape = ctx.tape, None  # activations freed as soon as the backward has run
        ctx.net.backward_from(dout, tape)
        return None, None, None, None, None


def net_apply(net, x_t, cond, t):
    """Run the HIP network; records the backward tape when a gradient is needed."""
    anchor = net.input_conv.weight
    if torch.is_grad_enabled() and anchor.requires_grad:
        return _NetFunction.apply(net, x_t, cond, t, anchor)
    return net.run_forward(x_t, cond, t, save=False)
