"""Per-kernel parity on the GPU: each HIP kernel vs a float64 CPU PyTorch evaluation of the same op.

fp32 kernels: relative L2 error < 1e-5 (parity mode); bf16 kernels: inputs are rounded to bf16
before the reference is evaluated, relative L2 < 1e-2 (bf16 output rounding + fp32 accumulation).
"""
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from cesm_emulator_amd import kernels as K
from cesm_emulator_amd import video_net as VN

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 1e-5, torch.bfloat16: 1e-2}


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b).clamp_min(1e-30)).item()


def to_cl(x):  # [B,C,F,H,W] -> [B*F,H,W,C]
    B, C, Fr, H, W = x.shape
    return x.permute(0, 2, 3, 4, 1).reshape(B * Fr, H, W, C).contiguous()


def from_cl(x, B):  # [B*F,H,W,C] -> [B,C,F,H,W]
    N, H, W, C = x.shape
    return x.reshape(B, N // B, H, W, C).permute(0, 4, 1, 2, 3).contiguous()


class PackHost:
    def _packed(self, w, cdt, cout, cin, kh, kw, swap, flip):
        return K.conv_pack(w.detach().contiguous(), cdt, cout, cin, kh, kw, swap, flip)


def make_rc(B, F, cdt):
    return VN.RunCtx(PackHost(), B, F, cdt, True)


def q(x, cdt):
    """round to the kernel storage dtype, return fp64 CPU copy"""
    return x.to(cdt).double().cpu()


CONV_CASES = [
    # kind, cin, cout, k, stride, pad
    ("conv", 64, 64, 3, 1, 1),
    ("conv", 128, 64, 3, 1, 1),
    ("conv", 64, 128, 3, 1, 1),
    ("conv", 64, 192, 1, 1, 0),
    ("conv", 64, 64, 4, 2, 1),
    ("convT", 64, 64, 4, 2, 1),
    ("convT", 128, 128, 4, 2, 1),
]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(dev, cdt, case):
    kind, cin, cout, k, s, p = case
    torch.manual_seed(0)
    B, Fr, H, W = 2, 3, 10, 14
    if kind == "conv":
        mod = nn.Conv3d(cin, cout, (1, k, k), (1, s, s), (0, p, p))
    else:
        mod = nn.ConvTranspose3d(cin, cout, (1, k, k), (1, s, s), (0, p, p))
    x = torch.randn(B, cin, Fr, H, W)
    mod_ref = mod.double()
    mod_dev = type(mod)(*([cin, cout, (1, k, k), (1, s, s), (0, p, p)])).to(dev)
    mod_dev.load_state_dict({kk: v.float() for kk, v in mod.state_dict().items()})
    rc = make_rc(B, Fr, cdt)
    spec = VN.ConvSpec(mod_dev)
    xd = to_cl(x).to(dev, cdt)
    y, st = VN.conv_forward(rc, spec, xd)
    xr = q(x, cdt).requires_grad_(True)
    wr = mod_ref.weight.detach().to(cdt).double().requires_grad_(True)
    br = mod_ref.bias.detach().double().requires_grad_(True)
    if kind == "conv":
        yr = F.conv3d(xr, wr, br, (1, s, s), (0, p, p))
    else:
        yr = F.conv_transpose3d(xr, wr, br, (1, s, s), (0, p, p))
    assert rel(from_cl(y, B), yr) < TOL[cdt]
    # backward
    g = torch.randn_like(yr)
    yr.backward(g.double())
    gd = to_cl(g.float()).to(dev, cdt)
    dx = VN.conv_backward(rc, spec, st, gd, True)
    torch.cuda.synchronize()
    gq = q(g, cdt)
    xr2 = q(x, cdt).requires_grad_(True)
    wr2 = wr.detach().clone().requires_grad_(True)
    br2 = br.detach().clone().requires_grad_(True)
    yr2 = (F.conv3d(xr2, wr2, br2, (1, s, s), (0, p, p)) if kind == "conv"
           else F.conv_transpose3d(xr2, wr2, br2, (1, s, s), (0, p, p)))
    yr2.backward(gq)
    assert rel(from_cl(dx, B), xr2.grad) < TOL[cdt]
    assert rel(mod_dev.weight.grad, wr2.grad) < TOL[cdt]
    assert rel(mod_dev.bias.grad, br2.grad) < TOL[cdt]


@pytest.mark.parametrize("cin,cout,k,st", [(256, 64, 1, 1), (64, 768, 1, 1), (64, 64, 4, 2), (128, 256, 1, 1)])
def test_wgrad_fused_bias(dev, cin, cout, k, st):
    """bias gradient produced inside the bf16 wide-tile wgrad (ones-operand MFMA, split-K partials) ==
    column sum of dY; the weight gradient is unchanged by it"""
    torch.manual_seed(9)
    Nb, H, W = 6, 37, 41
    pd = (k - 1) // 2 if k != 4 else 1
    Ho, Wo = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
    x = torch.randn(Nb, H, W, cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(Nb, Ho, Wo, cout, device=dev).to(torch.bfloat16)
    geom = (Ho, Wo, cout, k, k, st, pd, 1)
    dw1 = torch.zeros(cout, cin, 1, k, k, device=dev)
    dw2 = torch.zeros_like(dw1)
    db = torch.full((cout,), 0.5, device=dev)  # accumulates (+=)
    assert K.conv_wgrad(x, None, dy, None, dw1, geom, 0, 0, db=db)
    K.conv_wgrad(x, None, dy, None, dw2, geom, 0, 0)
    ref = dy.double().reshape(-1, cout).sum(0) + 0.5
    assert rel(db, ref) < 1e-5
    assert torch.equal(dw1, dw2)


@pytest.mark.parametrize("M,N,C", [(4000, 768, 256), (1237, 768, 512), (3001, 256, 128), (96 * 48 * 72, 768, 256),
                                   (5000, 64, 256), (96 * 48 * 72 + 5, 64, 256)])
def test_wgrad_square_tiles(dev, M, N, C):
    """1x1 weight gradient through the square-tile kernel (wgrad_sq_kernel, round 6: 256 x BN tiles, dY read once per
    row tile) vs float64, accumulating into a non-zero dW; pixel counts that leave partial steps and splits"""
    torch.manual_seed(11)
    x = torch.randn(1, 1, M, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(1, 1, M, N, device=dev).to(torch.bfloat16)
    assert K.conv_wgrad_variant(torch.bfloat16, 1, 1, M, C, 0, 1, M, N, N, 1, 1, 1, 0, 1).startswith("wgrad_sq_kernel")
    dw = torch.full((N, C, 1, 1), 0.25, device=dev)
    K.conv_wgrad(x, None, dy, None, dw, (1, M, N, 1, 1, 1, 0, 1), 0, 0)
    ref = dy.view(M, N).double().t() @ x.view(M, C).double() + 0.25
    err = rel(dw.view(N, C), ref)
    assert err < 1e-5, err


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_conv_pack_batch(dev, cdt):
    """cesm_conv_pack_batch (one launch for every cached weight pack, per-job (co, ci) tiles transposed through LDS)
    == cesm_conv_pack per job: 1x1 / 3x3 / 4x4 / 7x7 shapes, swap and flip, partial tiles in co and ci"""
    torch.manual_seed(5)
    geos = [(64, 64, 3, 3, 0, 0), (64, 64, 3, 3, 1, 1), (128, 64, 4, 4, 1, 1), (768, 64, 1, 1, 0, 0),
            (5, 7, 3, 3, 0, 1), (3, 1, 1, 1, 0, 0), (256, 512, 3, 3, 1, 1), (96, 40, 4, 4, 0, 0),
            (64, 2, 7, 7, 0, 0), (1, 64, 3, 3, 1, 1), (130, 100, 3, 3, 1, 0)]
    ws, outs, rows = [], [], []
    for (co, ci, kh, kw, swap, flip) in geos:
        w = torch.randn((ci, co, kh, kw) if swap else (co, ci, kh, kw), device=dev)
        out = torch.full((co * kh * kw * ci,), float("nan"), device=dev).to(cdt)
        ws.append(w)
        outs.append(out)
        rows.append([w.data_ptr(), out.data_ptr(), co, ci, kh, kw, swap, flip])
    tab, nblocks = K.conv_pack_table(rows, dev)
    assert nblocks == sum(K.pack_blocks(co, ci, kh, kw) for (co, ci, kh, kw, _, _) in geos)
    for grid in (nblocks, 3):  # any grid is correct (block-stride loop)
        for o in outs:
            o.fill_(float("nan"))
        K.conv_pack_batch(tab, len(rows), cdt, grid)
        for w, o, (co, ci, kh, kw, swap, flip) in zip(ws, outs, geos):
            ref = K.conv_pack(w, cdt, co, ci, kh, kw, swap, flip)
            assert torch.equal(o.view(-1), ref.view(-1)), (grid, co, ci, kh, kw, swap, flip)


def _pack_ref(w, cdt, co, ci, kh, kw, swap, flip):
    """torch restatement of the documented cesm_conv_pack layouts (include/cesm_hip.h): Wp[co][tap][ci], or the chunked
    form (bf16 3x3 / 4x4, Cout % 64 == 0, Cin % 32 == 0): element (co, tap, ci) at
    (((co/64 * Cin/32 + ci/32) * T + tap) * 64 + co%64) * 32 + ci%32"""
    g = w.transpose(0, 1) if swap else w  # [co][ci][kh][kw]
    if flip:
        g = g.flip(2, 3)
    g = g.reshape(co, ci, kh * kw).permute(0, 2, 1)  # [co][tap][ci]
    T = kh * kw
    if cdt == torch.bfloat16 and (kh, kw) in ((3, 3), (4, 4)) and co % 64 == 0 and ci % 32 == 0:
        g = g.reshape(co // 64, 64, T, ci // 32, 32).permute(0, 3, 2, 1, 4)  # [co/64][ci/32][tap][co%64][ci%32]
    return g.contiguous().reshape(-1).to(cdt)


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_conv_pack_layouts(dev, cdt):
    """cesm_conv_pack == the header's layout rule: row-major for fp32, 1x1, 7x7 and ragged channel counts; chunked
    for the bf16 3x3 / 4x4 packs the halo convs read (swap and flip included)"""
    torch.manual_seed(11)
    for (co, ci, kh, kw, swap, flip) in [(64, 64, 3, 3, 0, 0), (128, 64, 3, 3, 1, 1), (64, 96, 3, 3, 0, 1),
                                         (128, 128, 4, 4, 1, 1), (256, 64, 4, 4, 0, 0), (768, 64, 1, 1, 0, 0),
                                         (32, 64, 3, 3, 0, 0), (64, 40, 3, 3, 1, 1), (64, 2, 7, 7, 0, 0)]:
        w = torch.randn((ci, co, kh, kw) if swap else (co, ci, kh, kw), device=dev)
        got = K.conv_pack(w, cdt, co, ci, kh, kw, swap, flip)
        assert torch.equal(got.view(-1), _pack_ref(w, cdt, co, ci, kh, kw, swap, flip)), (co, ci, kh, kw, swap, flip)


@pytest.mark.parametrize("M,C", [(64, 64), (1000, 64), (40 * 77, 64), (6912 * 2 + 17, 128), (3000, 256), (777, 512)])
def test_qkv_bwd_fused(dev, M, C):
    """cesm_qkv_bwd (csrc/qkvbwd.hip: dqkv read once for dx and dW of the 768-channel to_qkv projection) against a
    float64 evaluation on the bf16-rounded operands and against the two-GEMM path it replaces (1x1 dgrad conv + wide
    weight-gradient GEMM); partial 64-pixel tiles, fewer tiles than streams (padding streams, zero slabs), every
    C slice count; dW accumulates (+=) and both outputs repeat bit for bit"""
    torch.manual_seed(M + C)
    dy = torch.randn(M, 768, device=dev).to(torch.bfloat16)
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    w = torch.randn(768, C, 1, 1, 1, device=dev) * C ** -0.5
    wt = K.conv_pack(w, torch.bfloat16, C, 768, 1, 1, 1, 1)
    assert K.qkv_bwd_supported(M, C)
    dw = torch.full((768, C), 0.5, device=dev)
    dx = K.qkv_bwd(dy, x, wt, dw)
    dw2 = torch.full((768, C), 0.5, device=dev)
    dx2 = K.qkv_bwd(dy, x, wt, dw2)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2)
    wq = w.reshape(768, C).to(torch.bfloat16).double()
    ref_dx = dy.double() @ wq
    ref_dw = dy.double().t() @ x.double()
    e_dx, e_dw = rel(dx, ref_dx), rel(dw - 0.5, ref_dw)
    # the path it replaces: dgrad 1x1 conv (gemm1x1) + conv_wgrad
    dx_ref = K.conv_fwd(dy.view(1, 1, M, 768), None, wt, None, (1, M, C, 1, 1, 1, 0, 1)).view(M, C)
    dw_ref = torch.zeros(768, C, 1, 1, 1, device=dev)
    K.conv_wgrad(x.view(1, 1, M, C), None, dy.view(1, 1, M, 768), None, dw_ref, (1, M, 768, 1, 1, 1, 0, 1), 0, 0)
    e_old_dx, e_old_dw = rel(dx, dx_ref), rel(dw - 0.5, dw_ref.view(768, C))
    print(f"qkv_bwd M={M} C={C}: dx {e_dx:.2e} dW {e_dw:.2e} vs float64; vs the two-GEMM path dx {e_old_dx:.2e} "
          f"dW {e_old_dw:.2e}")
    assert e_dx < 4e-3 and e_dw < 1e-5, (e_dx, e_dw)
    assert e_old_dx < 4e-3 and e_old_dw < 1e-5, (e_old_dx, e_old_dw)
    assert K.qkv_bwd(dy, x, wt, None).equal(dx)  # no weight gradient: the same dx


@pytest.mark.parametrize("H,W,cin,cout", [(12, 72, 64, 64), (8, 36, 128, 64), (6, 36, 64, 128), (10, 36, 256, 512), (20, 64, 128, 64)])
def test_conv3x3_tile_shapes_bf16(dev, H, W, cin, cout):
    """widths that are multiples of 36 take the 36-wide halo tiles (fwd/dgrad) and the 8 x 36 weight-
    gradient tiles; heights that are not tile multiples leave partial tile rows"""
    torch.manual_seed(3)
    cdt = torch.bfloat16
    B, Fr = 2, 2
    mod = nn.Conv3d(cin, cout, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    mod_dev = nn.Conv3d(cin, cout, (1, 3, 3), (1, 1, 1), (0, 1, 1)).to(dev)
    mod_dev.load_state_dict(mod.state_dict())
    x = torch.randn(B, cin, Fr, H, W)
    rc = make_rc(B, Fr, cdt)
    spec = VN.ConvSpec(mod_dev)
    y, st = VN.conv_forward(rc, spec, to_cl(x).to(dev, cdt))
    xr = q(x, cdt).requires_grad_(True)
    wr = mod.weight.detach().to(cdt).double().requires_grad_(True)
    br = mod.bias.detach().double().requires_grad_(True)
    yr = F.conv3d(xr, wr, br, 1, (0, 1, 1))
    assert rel(from_cl(y, B), yr) < TOL[cdt]
    g = torch.randn_like(yr)
    gq = q(g, cdt)
    yr.backward(gq)
    dx = VN.conv_backward(rc, spec, st, to_cl(g.float()).to(dev, cdt), True)
    torch.cuda.synchronize()
    assert rel(from_cl(dx, B), xr.grad) < TOL[cdt]
    assert rel(mod_dev.weight.grad, wr.grad) < TOL[cdt]
    assert rel(mod_dev.bias.grad, br.grad) < TOL[cdt]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_conv_concat_split_and_residual(dev, cdt):
    """two-source input (torch.cat fused into the loader), split dgrad + fused residual grads"""
    torch.manual_seed(1)
    B, Fr, H, W = 1, 2, 9, 11
    c1, c2, cout = 64, 128, 64
    mod = nn.Conv3d(c1 + c2, cout, (1, 3, 3), padding=(0, 1, 1))
    md = nn.Conv3d(c1 + c2, cout, (1, 3, 3), padding=(0, 1, 1)).to(dev)
    md.load_state_dict(mod.state_dict())
    a = torch.randn(B, c1, Fr, H, W)
    b = torch.randn(B, c2, Fr, H, W)
    res = torch.randn(B, cout, Fr, H, W)
    rc = make_rc(B, Fr, cdt)
    spec = VN.ConvSpec(md)
    y, st = VN.conv_forward(rc, spec, to_cl(a).to(dev, cdt), to_cl(b).to(dev, cdt), res=to_cl(res).to(dev, cdt))
    ar, br_ = q(a, cdt).requires_grad_(True), q(b, cdt).requires_grad_(True)
    wr = mod.weight.detach().to(cdt).double().requires_grad_(True)
    yr = F.conv3d(torch.cat([ar, br_], 1), wr, mod.bias.double(), padding=(0, 1, 1)) + q(res, cdt)
    assert rel(from_cl(y, B), yr) < TOL[cdt]
    g = torch.randn_like(yr)
    gq = q(g, cdt)
    yr.backward(gq)
    r1 = torch.randn(B, c1, Fr, H, W)
    r2 = torch.randn(B, c2, Fr, H, W)
    dx1, dx2 = VN.conv_backward(rc, spec, st, to_cl(g.float()).to(dev, cdt), True,
                                to_cl(r1).to(dev, cdt), to_cl(r2).to(dev, cdt))
    assert rel(from_cl(dx1, B), ar.grad + q(r1, cdt)) < TOL[cdt]
    assert rel(from_cl(dx2, B), br_.grad + q(r2, cdt)) < TOL[cdt]
    assert rel(md.weight.grad, wr.grad) < TOL[cdt]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("with_ss", [True, False])
@pytest.mark.parametrize("cout", [128, 512])
def test_block_groupnorm(dev, cdt, with_ss, cout):
    """Block: conv -> GroupNorm(8) -> x*(scale+1)+shift -> SiLU (+residual), fwd and bwd (incl. the conv
    bias gradient produced by the GroupNorm backward's reduction)"""
    torch.manual_seed(2)
    B, Fr, H, W, cin = 2, 3, 8, 12, 64
    blk = VN.Block(cin, cout).to(dev)
    with torch.no_grad():
        blk.norm.weight.uniform_(0.5, 1.5)
        blk.norm.bias.uniform_(-0.5, 0.5)
    x = torch.randn(B, cin, Fr, H, W)
    ss = torch.randn(B, 2 * cout) * 0.3 if with_ss else None
    res = torch.randn(B, cout, Fr, H, W)
    rc = make_rc(B, Fr, cdt)
    out, st = VN.block_fwd(rc, blk, to_cl(x).to(dev, cdt), None, None if ss is None else ss.to(dev),
                           to_cl(res).to(dev, cdt))
    # reference
    xr = q(x, cdt).requires_grad_(True)
    wr = blk.proj.weight.detach().cpu().to(cdt).double().requires_grad_(True)
    bconv = blk.proj.bias.detach().cpu().double().requires_grad_(True)
    gam = blk.norm.weight.detach().cpu().double().requires_grad_(True)
    bet = blk.norm.bias.detach().cpu().double().requires_grad_(True)
    ssr = ss.double().requires_grad_(True) if ss is not None else None
    y = F.conv3d(xr, wr, bconv, padding=(0, 1, 1))
    y = q(y.detach(), cdt).requires_grad_(True) if cdt == torch.bfloat16 else y  # kernel stores y in cdt
    h = F.group_norm(y, 8, gam, bet, 1e-5)
    if ssr is not None:
        sc, sh = ssr[:, :cout, None, None, None], ssr[:, cout:, None, None, None]
        h = h * (sc + 1) + sh
    o = F.silu(h) + q(res, cdt)
    assert rel(from_cl(out, B), o) < TOL[cdt] * (3 if cdt == torch.bfloat16 else 1)
    g = torch.randn_like(o)
    o.backward(q(g, cdt))
    dx, dss = VN.block_bwd(rc, blk, st, to_cl(g.float()).to(dev, cdt), ssr is not None)
    tol = TOL[cdt] * (5 if cdt == torch.bfloat16 else 10)
    assert rel(blk.norm.weight.grad, gam.grad) < tol
    assert rel(blk.norm.bias.grad, bet.grad) < tol
    ref_db = bconv.grad if cdt == torch.float32 else y.grad.sum((0, 2, 3, 4))
    assert rel(blk.proj.bias.grad, ref_db) < tol
    if ssr is not None:
        assert rel(dss, ssr.grad) < tol
    if cdt == torch.float32:
        assert rel(from_cl(dx, B), xr.grad) < tol
        assert rel(blk.proj.weight.grad, wr.grad) < tol


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [64, 256, 512])
def test_layernorm(dev, cdt, C):
    torch.manual_seed(3)
    V = 1000
    x = torch.randn(V, C) * 2 + 0.5
    gamma = torch.rand(C) + 0.5
    out, mr = K.ln_fwd(x.to(dev, cdt).contiguous(), gamma.to(dev))
    xr = q(x, cdt).requires_grad_(True)
    gr = gamma.double().requires_grad_(True)
    mu = xr.mean(-1, keepdim=True)
    var = ((xr - mu) ** 2).mean(-1, keepdim=True)
    o = (xr - mu) / torch.sqrt(var + 1e-5) * gr
    assert rel(out, o) < TOL[cdt]
    g = torch.randn(V, C)
    dres = torch.randn(V, C)
    o.backward(q(g, cdt))
    dgam = torch.zeros(C, device=dev)
    dx = K.ln_bwd(g.to(dev, cdt).contiguous(), x.to(dev, cdt).contiguous(), mr, gamma.to(dev), dgam,
                  dres=dres.to(dev, cdt).contiguous())
    assert rel(dx, xr.grad + q(dres, cdt)) < TOL[cdt] * 2
    assert rel(dgam, gr.grad) < TOL[cdt] * 2


def _tattn_ref(qkv, bias, freqs, B, Fr, HW, scale):
    """oracle-style temporal attention core on qkv [B*F*HW, 768] (float64)"""
    x = qkv.view(B, Fr, HW, 3, 8, 32).permute(3, 0, 2, 4, 1, 5)  # 3, B, HW, h, F, d
    qq, kk, vv = x[0] * scale, x[1], x[2]
    pos = torch.arange(Fr, dtype=torch.float64)
    ang = (pos[:, None] * freqs.double()[None, :]).repeat_interleave(2, -1)

    def rot(t):
        t2 = t.unflatten(-1, (-1, 2))
        rh = torch.stack((-t2[..., 1], t2[..., 0]), -1).flatten(-2)
        return t * ang.cos() + rh * ang.sin()

    qq, kk = rot(qq), rot(kk)
    sim = torch.einsum("bphid,bphjd->bphij", qq, kk) + bias.double()
    sim = sim - sim.amax(-1, keepdim=True)
    o = torch.einsum("bphij,bphjd->bphid", sim.softmax(-1), vv)  # B, HW, h, F, d
    return o.permute(0, 3, 1, 2, 4).reshape(B * Fr * HW, 256)


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Fr", [1, 3, 12, 33, 64, 80, 100, 120])
def test_temporal_attention_core(dev, cdt, Fr):
    """unfused temporal attention; F > 32 exercises the F-sized LDS tables (decadal window F = 120)"""
    torch.manual_seed(4)
    B, HW = 2, (77 if Fr <= 32 else 13)
    qkv = torch.randn(B * Fr * HW, 768)
    table = torch.randn(32, 8)
    freqs = 1.0 / (10000 ** (torch.arange(0, 32, 2).float() / 32))
    scale = 32 ** -0.5
    bias = K.relpos_fwd(table.to(dev), Fr)
    from oracle.ref_cpu import RelativePositionBias
    rp = RelativePositionBias(8, 32, 32)
    rp.relative_attention_bias.weight.data.copy_(table)
    bias_ref = rp(Fr)
    assert torch.equal(bias.cpu(), bias_ref)
    rot = K.rope_table(freqs.to(dev), Fr)
    qd = qkv.to(dev, cdt).contiguous()
    out, lse = K.tattn_fwd(qd, bias, rot, B, Fr, HW, scale)
    qr = q(qkv, cdt).requires_grad_(True)
    br = bias_ref.detach().double().requires_grad_(True)
    o = _tattn_ref(qr, br, freqs, B, Fr, HW, scale)
    assert rel(out, o) < TOL[cdt] * 2
    g = torch.randn_like(o)
    o.backward(q(g, cdt))
    dtable = torch.zeros(32, 8, device=dev)
    dqkv = K.tattn_bwd(qd, out, g.to(dev, cdt).contiguous(), lse, bias, rot, dtable, B, Fr, HW, scale)
    tol = TOL[cdt] * (3 if cdt == torch.bfloat16 else 10)
    assert rel(dqkv, qr.grad) < tol
    # table grad: scatter of bias grad through the bucket map
    tbl = table.double().requires_grad_(True)
    rp2 = RelativePositionBias(8, 32, 32).double()
    rp2.relative_attention_bias.weight.data.copy_(tbl.detach())
    bref = rp2(Fr)
    (bref * br.grad).sum().backward()
    assert rel(dtable, rp2.relative_attention_bias.weight.grad) < tol


def test_tflash_long_window_full_grid(dev):
    """the MFMA flash core at config 4's level-0 size (F = 120, 192x288, B = 1): the query / output tiles of the
    late frames sit > 2^32 B past the tile base, so a tile resource spanning every remaining frame wrapped its
    32-bit num_records and dropped rows.  Attention is per pixel, so the float64 reference (and the
    dq / dk / dv it implies) is evaluated on a sample of pixels only (video_net.py:403-454)."""
    torch.manual_seed(7)
    B, Fr, HW = 1, 120, 192 * 288
    scale = 32 ** -0.5
    freqs = 1.0 / (10000 ** (torch.arange(0, 32, 2).float() / 32))
    table = torch.randn(32, 8)
    bias = K.relpos_fwd(table.to(dev), Fr)
    rot = K.rope_table(freqs.to(dev), Fr)
    qd = torch.randn(B * Fr * HW, 768, device=dev, dtype=torch.bfloat16)
    out, lse = K.tattn_fwd(qd, bias, rot, B, Fr, HW, scale)
    g = torch.randn(B * Fr * HW, 256, device=dev, dtype=torch.bfloat16)
    dqkv = K.tattn_bwd(qd, out, g, lse, bias, rot, None, B, Fr, HW, scale)
    torch.cuda.synchronize()
    pix = torch.cat([torch.tensor([0, 1, HW // 2, HW - 1]), torch.randint(0, HW, (60,))]).to(dev)
    npx = pix.numel()

    def take(t):  # [B*F*HW, c] -> float64 CPU [B*F*npx, c] (the sampled pixels as a small grid)
        return t.view(B, Fr, HW, -1)[:, :, pix].reshape(B * Fr * npx, -1).double().cpu()

    qr = take(qd).requires_grad_(True)
    o = _tattn_ref(qr, bias.double().cpu(), freqs, B, Fr, npx, scale)
    assert torch.isfinite(out).all()
    assert rel(take(out), o) < 2e-2
    o.backward(take(g))
    assert rel(take(dqkv), qr.grad) < 3e-2
    # every frame of the late query tiles carries signal (the wrapped resource returned zero rows there)
    per_frame = take(out).view(Fr, npx, 256).abs().sum((1, 2))
    assert (per_frame > 0).all()


def _sla_ref(qkv, Nf, HW, scale):
    x = qkv.view(Nf, HW, 3, 8, 32).permute(2, 0, 3, 4, 1)  # 3, Nf, h, d, n
    qq = x[0].softmax(dim=-2) * scale
    kk = x[1].softmax(dim=-1)
    ctx = torch.einsum("bhdn,bhen->bhde", kk, x[2])
    out = torch.einsum("bhde,bhdn->bhen", ctx, qq)  # Nf, h, e, n
    return out.permute(0, 3, 1, 2).reshape(Nf * HW, 256)


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("HW", [77, 3000])
def test_spatial_linear_attention_core(dev, cdt, HW):
    torch.manual_seed(5)
    Nf = 3
    qkv = torch.randn(Nf * HW, 768) * 2
    scale = 32 ** -0.5
    qd = qkv.to(dev, cdt).contiguous()
    out, ctx, ml = K.sla_fwd(qd, Nf, HW, scale)
    qr = q(qkv, cdt).requires_grad_(True)
    o = _sla_ref(qr, Nf, HW, scale)
    assert rel(out, o) < TOL[cdt] * 2
    g = torch.randn_like(o)
    o.backward(q(g, cdt))
    dqkv = K.sla_bwd(qd, g.to(dev, cdt).contiguous(), ctx, ml, Nf, HW, scale)
    assert rel(dqkv, qr.grad) < TOL[cdt] * (3 if cdt == torch.bfloat16 else 10)


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Fx", [1, 3])
def test_stem_and_head(dev, cdt, Fx):
    torch.manual_seed(6)
    B, Fr, H, W = 2, 3, 20, 35
    conv = nn.Conv3d(2, 64, (1, 7, 7), padding=(0, 3, 3))
    cd = nn.Conv3d(2, 64, (1, 7, 7), padding=(0, 3, 3)).to(dev)
    cd.load_state_dict(conv.state_dict())
    xt = torch.randn(B, Fx, H, W)
    cond = torch.randn(B, Fr, H, W)
    y = K.stem_fwd(xt.to(dev), cond.to(dev), cd.weight, cd.bias, Fr, cdt)
    xin = torch.cat([xt[:, None].expand(B, 1, Fr, H, W), cond[:, None]], 1).double()
    wr = conv.weight.detach().double().requires_grad_(True)
    yr = F.conv3d(xin, wr, conv.bias.double(), padding=(0, 3, 3))
    assert rel(from_cl(y, B), yr) < TOL[cdt]
    g = torch.randn_like(yr)
    yr.backward(q(g, cdt))
    dw = torch.zeros_like(cd.weight)
    K.stem_wgrad(xt.to(dev), cond.to(dev), to_cl(g.float()).to(dev, cdt), dw, Fr)
    assert rel(dw, wr.grad) < TOL[cdt]
    # head: Conv3d(64->1, 1) on frame F//2
    hw = torch.randn(64)
    hb = torch.randn(1)
    x = torch.randn(B, 64, Fr, H, W)
    out = K.head_fwd(to_cl(x).to(dev, cdt), hw.to(dev), hb.to(dev), B, Fr)
    xr = q(x, cdt).requires_grad_(True)
    hwr = hw.double().requires_grad_(True)
    ref = (xr[:, :, Fr // 2] * hwr[None, :, None, None]).sum(1, keepdim=True) + hb.double()
    assert rel(out, ref) < TOL[cdt]
    go = torch.randn_like(ref)
    ref.backward(go)
    dwh = torch.zeros(64, device=dev)
    dbh = torch.zeros(1, device=dev)
    dx = K.head_bwd(go.float().to(dev).contiguous(), to_cl(x).to(dev, cdt), hw.to(dev), dwh, dbh, B, Fr)
    assert rel(from_cl(dx, B), xr.grad) < TOL[cdt]
    assert rel(dwh, hwr.grad) < TOL[cdt]
    assert abs(dbh.item() - go.sum().item()) < 1e-3


def test_small_linear_and_time_emb(dev):
    torch.manual_seed(7)
    R, I, O = 5, 64, 96
    x = torch.randn(R, I)
    w = torch.randn(O, I) * 0.1
    b = torch.randn(O)
    for silu in (False, True):
        y = K.linear_small(x.to(dev), w.to(dev), b.to(dev), silu)
        xr = x.double().requires_grad_(True)
        wr = w.double().requires_grad_(True)
        br = b.double().requires_grad_(True)
        yr = F.linear(F.silu(xr) if silu else xr, wr, br)
        assert rel(y, yr) < 1e-6
        g = torch.randn(R, O)
        yr.backward(g.double())
        dx = torch.zeros(R, I, device=dev)
        dw = torch.zeros(O, I, device=dev)
        db = torch.zeros(O, device=dev)
        K.linear_small_bwd(x.to(dev), w.to(dev), g.to(dev), dx, dw, db, silu, True)
        assert rel(dx, xr.grad) < 1e-6 and rel(dw, wr.grad) < 1e-6 and rel(db, br.grad) < 1e-6
    t = torch.tensor([0, 1, 17, 999])
    emb = K.sinusoidal(t.to(dev), 64)
    from oracle.ref_cpu import SinusoidalPosEmb
    assert rel(emb, SinusoidalPosEmb(64)(t)) < 1e-5


def test_adamw_clip_matches_torch(dev):
    from cesm_emulator_amd.optim import FusedAdamW
    torch.manual_seed(8)
    ps = [torch.randn(37, 5), torch.randn(1000), torch.randn(3, 3, 3)]
    gs = [[torch.randn_like(p) * 3 for p in ps] for _ in range(3)]
    ref = [p.clone().double().requires_grad_(True) for p in ps]
    opt_r = torch.optim.AdamW(ref, lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4)
    dp = [nn.Parameter(p.clone().to(dev)) for p in ps]
    opt = FusedAdamW(dp, lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_grad_norm=1.0)
    for step in range(3):
        for r, g in zip(ref, gs[step]):
            r.grad = g.double().clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt_r.step()
        opt.zero_grad()
        for p, g in zip(dp, gs[step]):
            p.grad.copy_(g.to(dev))
        opt.step()
    for p, r in zip(dp, ref):
        assert rel(p.detach(), r.detach()) < 1e-6


def test_q_sample_mse(dev):
    from cesm_emulator_amd.model import Diffusion
    from oracle.ref_cpu import Diffusion as RD
    torch.manual_seed(9)
    d = Diffusion(nn.Identity()).to(dev)
    rd = RD(nn.Identity())
    for name, buf in rd.named_buffers():
        assert torch.equal(buf, getattr(d, name).cpu()), name
    x0 = torch.randn(3, 1, 16, 24)
    noise = torch.randn_like(x0)
    t = torch.tensor([0, 500, 999])
    xt, _ = d.q_sample(x0.to(dev), t.to(dev), noise.to(dev))
    xr, _ = rd.q_sample(x0, t, noise)
    assert rel(xt, xr) < 1e-6
    pred = torch.randn_like(x0)
    loss = K.mse(pred.to(dev), noise.to(dev))
    assert abs(loss.item() - F.mse_loss(pred, noise).item()) < 1e-6


def test_window_gather(dev):
    """device gather == WindowedAllMembersDataset_random.__getitem__ semantics (host restatement)"""
    from oracle.ref_data import window_item as host_window_item
    torch.manual_seed(10)
    T, M, H, W, Kw = 9, 3, 10, 12, 5
    cond = torch.randn(T, M, H, W)
    tgt = torch.randn(T, M, H, W)
    items = torch.tensor([[0, 1, 2, 0, 1, 2], [3, 2, 5, 1, 0, 0], [4, 0, 6, 1, 2, 3]], dtype=torch.int64)
    cw, x0 = K.window_gather(cond.to(dev), tgt.to(dev), items.to(dev), Kw, 7, 8, True)
    for i in range(items.shape[0]):
        c_ref, x_ref = host_window_item(cond.numpy(), tgt.numpy(), items[i].tolist(), Kw, 7, 8, True)
        assert torch.equal(cw[i].cpu(), torch.from_numpy(c_ref))
        assert torch.equal(x0[i].cpu(), torch.from_numpy(x_ref))


@pytest.mark.parametrize("C", [64, 128, 256, 512])
@pytest.mark.parametrize("Fr", [1, 3, 12])
def test_fused_temporal_block_forward(dev, C, Fr):
    """cesm_tblock_fwd (LN+QKV+RoPE+MFMA core+out-proj+residual in one kernel) vs a float64
    evaluation of the reference block on the same bf16-rounded inputs/weights"""
    torch.manual_seed(11)
    B, H, W = 2, 5, 7
    rot_mod = VN.RotaryEmbedding(32)
    res_mod = VN.Residual(VN.PreNorm(C, VN.EinopsToAndFrom(VN.Attention(C, 8, 32, rot_mod)))).to(dev)
    with torch.no_grad():
        res_mod.fn.norm.gamma.uniform_(0.5, 1.5)
    attn = res_mod.fn.fn.fn
    x = torch.randn(B, C, Fr, H, W)
    table = torch.randn(32, 8)
    rc = make_rc(B, Fr, torch.bfloat16)
    rc.bias = K.relpos_fwd(table.to(dev), Fr)
    rc.rot = K.rope_table(rot_mod.freqs.to(dev), Fr)
    xd = to_cl(x).to(dev, torch.bfloat16)
    wq = K.conv_pack(attn.to_qkv.weight.detach(), torch.bfloat16, 768, C, 1, 1, 0, 0)
    wo = K.conv_pack(attn.to_out.weight.detach(), torch.bfloat16, C, 256, 1, 1, 0, 0)
    y, mr, lse, _ = K.tblock_fwd(xd, res_mod.fn.norm.gamma.reshape(-1), wq, wo, rc.bias, rc.rot, B, Fr, attn.scale)
    # float64 reference (oracle module) on bf16-rounded x and weights
    from oracle import ref_cpu as R
    ref = R.Residual(R.PreNorm(C, R.EinopsToAndFrom(R.Attention(C, 8, 32, R.RotaryEmbedding(32))))).double()
    ref.fn.norm.gamma.data.copy_(res_mod.fn.norm.gamma.detach().cpu().double())
    ref.fn.fn.fn.to_qkv.weight.data.copy_(attn.to_qkv.weight.detach().cpu().to(torch.bfloat16).double())
    ref.fn.fn.fn.to_out.weight.data.copy_(attn.to_out.weight.detach().cpu().to(torch.bfloat16).double())
    rp = R.RelativePositionBias(8, 32, 32)
    rp.relative_attention_bias.weight.data.copy_(table)
    with torch.no_grad():
        yr = ref(q(x, torch.bfloat16), pos_bias=rp(Fr).double())
    err = rel(from_cl(y, B), yr)
    print(f"fused tblock C={C} F={Fr}: rel {err:.2e}")
    assert err < 2e-2
    # saved LN stats match
    xv = q(x, torch.bfloat16).permute(0, 2, 3, 4, 1).reshape(-1, C)
    torch.testing.assert_close(mr[:, 0].cpu().double(), xv.mean(1), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("C", [64, 128, 256, 512])
@pytest.mark.parametrize("Fr", [1, 5, 12])
def test_fused_temporal_block_backward(dev, C, Fr):
    """cesm_tblock_bwd (recompute + MFMA core backward + LN backward in one kernel) and the weight
    gradients built from its dqkv/o/xn outputs vs float64 autograd through the reference block"""
    torch.manual_seed(12)
    B, H, W = 2, 5, 7
    rot_mod = VN.RotaryEmbedding(32)
    res_mod = VN.Residual(VN.PreNorm(C, VN.EinopsToAndFrom(VN.Attention(C, 8, 32, rot_mod)))).to(dev)
    with torch.no_grad():
        res_mod.fn.norm.gamma.uniform_(0.5, 1.5)
    attn = res_mod.fn.fn.fn
    x = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    g = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    table = torch.randn(32, 8)
    rc = make_rc(B, Fr, torch.bfloat16)
    rc.bias = K.relpos_fwd(table.to(dev), Fr)
    rc.rot = K.rope_table(rot_mod.freqs.to(dev), Fr)
    xd = to_cl(x).to(dev, torch.bfloat16)
    gd = to_cl(g).to(dev, torch.bfloat16)
    wqkv, wout = attn.to_qkv.weight.detach(), attn.to_out.weight.detach()
    wq = K.conv_pack(wqkv, torch.bfloat16, 768, C, 1, 1, 0, 0)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wq_t = K.conv_pack(wqkv, torch.bfloat16, C, 768, 1, 1, 1, 1)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    gamma = res_mod.fn.norm.gamma.detach().reshape(-1).contiguous()
    save_o = C <= 256
    _, mr, lse, o_fwd = K.tblock_fwd(xd, gamma, wq, wo, rc.bias, rc.rot, B, Fr, attn.scale, save_o=save_o)
    dgamma = torch.zeros(C, device=dev)
    dtable = torch.zeros(32, 8, device=dev)
    dx, dqkv, o, xn = K.tblock_bwd(xd, gd, gamma, mr, lse, wq, wq_t, wo_t, rc.bias, rc.rot, dgamma, dtable, B, Fr,
                                   attn.scale)
    if save_o:  # the forward's O (what training uses for dW_out) == the backward's recomputed emission
        assert rel(o_fwd, o) < 1e-2
        # and the backward without the O emission gives the same dx / dqkv
        dg2, dt2 = torch.zeros(C, device=dev), torch.zeros(32, 8, device=dev)
        dx2, dqkv2, o2, _ = K.tblock_bwd(xd, gd, gamma, mr, lse, wq, wq_t, wo_t, rc.bias, rc.rot, dg2, dt2, B, Fr,
                                         attn.scale, emit_o=False)
        dg3, dt3 = torch.zeros(C, device=dev), torch.zeros(32, 8, device=dev)
        dx3, dqkv3, _, _ = K.tblock_bwd(xd, gd, gamma, mr, lse, wq, wq_t, wo_t, rc.bias, rc.rot, dg3, dt3, B, Fr,
                                        attn.scale)
        print("rerun identical:", torch.equal(dx3, dx), torch.equal(dqkv3, dqkv), " no-emit identical:",
              torch.equal(dx2, dx), torch.equal(dqkv2, dqkv), " max |ddx|", (dx2.float() - dx.float()).abs().max().item())
        assert o2 is None and rel(dx2, dx) < 1e-2 and rel(dqkv2, dqkv) < 1e-2
        o = o_fwd
    dwq = dqkv.reshape(-1, 768).double().t() @ xn.reshape(-1, C).double()
    dwo = gd.reshape(-1, C).double().t() @ o.reshape(-1, 256).double()
    # float64 reference
    from oracle import ref_cpu as R
    ref = R.Residual(R.PreNorm(C, R.EinopsToAndFrom(R.Attention(C, 8, 32, R.RotaryEmbedding(32))))).double()
    ref.fn.norm.gamma.data.copy_(gamma.cpu().double().view_as(ref.fn.norm.gamma))
    ref.fn.fn.fn.to_qkv.weight.data.copy_(wqkv.cpu().to(torch.bfloat16).double())
    ref.fn.fn.fn.to_out.weight.data.copy_(wout.cpu().to(torch.bfloat16).double())
    rp = R.RelativePositionBias(8, 32, 32).double()
    rp.relative_attention_bias.weight.data.copy_(table.double())
    xr = x.double().requires_grad_(True)
    yr = ref(xr, pos_bias=rp(Fr))
    (yr * g.double()).sum().backward()
    errs = {
        "dx": rel(from_cl(dx, B), xr.grad),
        "dgamma": rel(dgamma.double(), ref.fn.norm.gamma.grad.reshape(-1)),
        "dtable": rel(dtable.double(), rp.relative_attention_bias.weight.grad),
        "dWqkv": rel(dwq, ref.fn.fn.fn.to_qkv.weight.grad),
        "dWout": rel(dwo, ref.fn.fn.fn.to_out.weight.grad),
    }
    print(f"fused tblock bwd C={C} F={Fr}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v < 3e-2, (k, v)


def _sla_block(C, dev):
    res = VN.Residual(VN.PreNorm(C, VN.SpatialLinearAttention(C, 8, 32))).to(dev)
    with torch.no_grad():
        res.fn.norm.gamma.uniform_(0.5, 1.5)
        res.fn.fn.to_out.bias.uniform_(-0.1, 0.1)
    return res


def _sla_block_ref(res, C):
    from oracle import ref_cpu as R
    ref = R.Residual(R.PreNorm(C, R.SpatialLinearAttention(C, heads=8, dim_head=32))).double()
    sla = res.fn.fn
    ref.fn.norm.gamma.data.copy_(res.fn.norm.gamma.detach().cpu().double())
    ref.fn.fn.to_qkv.weight.data.copy_(sla.to_qkv.weight.detach().cpu().to(torch.bfloat16).double())
    ref.fn.fn.to_out.weight.data.copy_(sla.to_out.weight.detach().cpu().to(torch.bfloat16).double())
    ref.fn.fn.to_out.bias.data.copy_(sla.to_out.bias.detach().cpu().double())
    return ref


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("H,W", [(8, 8), (12, 20), (37, 29)])
def test_fused_sla_forward(dev, H, W, C):
    """cesm_slaf_fwd (LN + online-softmax context + output projection, no per-pixel intermediates)
    vs a float64 evaluation of the reference block on bf16-rounded inputs/weights"""
    torch.manual_seed(13)
    B, Fr = 2, 3
    res = _sla_block(C, dev)
    sla = res.fn.fn
    x = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    xd = to_cl(x).to(dev, torch.bfloat16)
    wq = K.conv_pack(sla.to_qkv.weight.detach().reshape(768, C), torch.bfloat16, 768, C, 1, 1, 0, 0)
    wo = K.conv_pack(sla.to_out.weight.detach().reshape(C, 256), torch.bfloat16, C, 256, 1, 1, 0, 0)
    y, st = K.slaf_fwd(xd, res.fn.norm.gamma.detach().reshape(-1).contiguous(), wq, wo, sla.to_out.bias.detach(),
                       sla.scale)
    ref = _sla_block_ref(res, C)
    with torch.no_grad():
        yr = ref(x)
    err = rel(from_cl(y, B), yr)
    # the context itself: ctx[n][h][d][e]
    xr = x.permute(0, 2, 1, 3, 4).reshape(B * Fr, C, H * W)
    mu = xr.mean(1, keepdim=True)
    var = xr.var(1, unbiased=False, keepdim=True)
    xn = (xr - mu) / (var + 1e-5).sqrt() * ref.fn.norm.gamma.reshape(1, C, 1)
    qkv = torch.einsum("oc,ncp->nop", ref.fn.fn.to_qkv.weight.reshape(768, C), xn)
    k = qkv[:, 256:512].reshape(B * Fr, 8, 32, H * W).softmax(-1)
    v = qkv[:, 512:].reshape(B * Fr, 8, 32, H * W)
    ctx = torch.einsum("nhdp,nhep->nhde", k, v)
    cerr = rel(st[1], ctx)
    print(f"fused sla fwd HxW={H}x{W}: y rel {err:.2e} ctx rel {cerr:.2e}")
    assert cerr < 2e-2
    assert err < 2e-2


@pytest.mark.parametrize("save_o", [False, True])
@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("H,W", [(8, 8), (12, 20), (37, 29)])
def test_fused_sla_backward(dev, H, W, C, save_o):
    """cesm_slaf_bwd (+ weight gradients from its dqkv/o/xn outputs) vs float64 autograd through the
    reference SpatialLinearAttention block; save_o: O written by the forward instead of the backward"""
    torch.manual_seed(14)
    B, Fr = 2, 3
    res = _sla_block(C, dev)
    sla = res.fn.fn
    x = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    g = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    xd = to_cl(x).to(dev, torch.bfloat16)
    gd = to_cl(g).to(dev, torch.bfloat16)
    wqkv = sla.to_qkv.weight.detach().reshape(768, C)
    wout = sla.to_out.weight.detach().reshape(C, 256)
    wq = K.conv_pack(wqkv, torch.bfloat16, 768, C, 1, 1, 0, 0)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wq_t = K.conv_pack(wqkv, torch.bfloat16, C, 768, 1, 1, 1, 1)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    gamma = res.fn.norm.gamma.detach().reshape(-1).contiguous()
    _, st = K.slaf_fwd(xd, gamma, wq, wo, sla.to_out.bias.detach(), sla.scale, save_o=save_o)
    dgamma = torch.zeros(C, device=dev)
    dx, dqkv, o, xn = K.slaf_bwd(xd, gd, gamma, wq, wq_t, wo_t, st, dgamma, sla.scale)
    if save_o:  # the forward's O equals the one the backward emits (same bf16 rounding up to 1 ulp)
        _, st2 = K.slaf_fwd(xd, gamma, wq, wo, sla.to_out.bias.detach(), sla.scale)
        _, _, o_bwd, _ = K.slaf_bwd(xd, gd, gamma, wq, wq_t, wo_t, st2, torch.zeros(C, device=dev), sla.scale)
        assert rel(o, o_bwd) < 1e-2
    dwq = dqkv.reshape(-1, 768).double().t() @ xn.reshape(-1, C).double()
    dwo = gd.reshape(-1, C).double().t() @ o.reshape(-1, 256).double()
    ref = _sla_block_ref(res, C)
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    (yr * g.double()).sum().backward()
    errs = {
        "dx": rel(from_cl(dx, B), xr.grad),
        "dgamma": rel(dgamma.double(), ref.fn.norm.gamma.grad.reshape(-1)),
        "dWqkv": rel(dwq, ref.fn.fn.to_qkv.weight.grad.reshape(768, C)),
        "dWout": rel(dwo, ref.fn.fn.to_out.weight.grad.reshape(C, 256)),
    }
    print(f"fused sla bwd HxW={H}x{W}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v < 3e-2, (k, v)


@pytest.mark.parametrize("Fr", [1, 5, 12])
@pytest.mark.parametrize("B,H,W", [(2, 5, 7), (1, 12, 16), (3, 9, 13)])
def test_tblock_fold_forward_and_dw_backward(dev, Fr, B, H, W):
    """cesm_tblock_fwd_fold + cesm_tblock_bwd_dw (head-parallel backward with in-kernel dW_qkv / dgamma, no
    dqkv / xn intermediates; the level-0 training path at C = 64) vs float64 autograd through the
    reference block (video_net.py:368-454 under Residual(PreNorm)); pixel counts that leave partial
    4-pixel groups, groups spanning samples"""
    C = 64
    torch.manual_seed(21)
    rot_mod = VN.RotaryEmbedding(32)
    res_mod = VN.Residual(VN.PreNorm(C, VN.EinopsToAndFrom(VN.Attention(C, 8, 32, rot_mod)))).to(dev)
    with torch.no_grad():
        res_mod.fn.norm.gamma.uniform_(0.5, 1.5)
    attn = res_mod.fn.fn.fn
    assert K.tblock_bwd_dw_supported(B, Fr, H * W, C)
    x = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    g = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    table = torch.randn(32, 8)
    rc = make_rc(B, Fr, torch.bfloat16)
    rc.bias = K.relpos_fwd(table.to(dev), Fr)
    rc.rot = K.rope_table(rot_mod.freqs.to(dev), Fr)
    xd = to_cl(x).to(dev, torch.bfloat16)
    gd = to_cl(g).to(dev, torch.bfloat16)
    wqkv = attn.to_qkv.weight.detach().contiguous()
    wout = attn.to_out.weight.detach()
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    gamma = res_mod.fn.norm.gamma.detach().reshape(-1).contiguous()
    y, mr, lse, o = K.tblock_fwd_fold(xd, gamma, wqkv, wo, rc.bias, rc.rot, B, Fr, attn.scale, save_o=True)
    dgamma = torch.full((C,), 0.25, device=dev)   # accumulates (+=)
    dtable = torch.zeros(32, 8, device=dev)
    dwq = torch.full((768, C), 0.5, device=dev)   # accumulates (+=)
    dx, ob = K.tblock_bwd_dw(xd, gd, mr, lse, wqkv, gamma, wo_t, rc.bias, rc.rot, dwq, dgamma, dtable, B, Fr,
                             attn.scale, emit_o=True)
    # the O emission (round 6: the backward recomputes O = P V for the to_out weight gradient) leaves dx unchanged
    dx2 = K.tblock_bwd_dw(xd, gd, mr, lse, wqkv, gamma, wo_t, rc.bias, rc.rot, None, None, None, B, Fr, attn.scale)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx2)
    # the to_out weight gradient from the backward's O (what the training path uses)
    dwo = gd.reshape(-1, C).double().t() @ ob.reshape(-1, 256).double()
    from oracle import ref_cpu as R
    ref = R.Residual(R.PreNorm(C, R.EinopsToAndFrom(R.Attention(C, 8, 32, R.RotaryEmbedding(32))))).double()
    ref.fn.norm.gamma.data.copy_(gamma.cpu().double().view_as(ref.fn.norm.gamma))
    ref.fn.fn.fn.to_qkv.weight.data.copy_(wqkv.cpu().double())
    ref.fn.fn.fn.to_out.weight.data.copy_(wout.cpu().to(torch.bfloat16).double())
    rp = R.RelativePositionBias(8, 32, 32).double()
    rp.relative_attention_bias.weight.data.copy_(table.double())
    xr = x.double().requires_grad_(True)
    yr = ref(xr, pos_bias=rp(Fr))
    (yr * g.double()).sum().backward()
    errs = {
        "y": rel(from_cl(y, B), yr.detach()),
        "dx": rel(from_cl(dx, B), xr.grad),
        "dgamma": rel(dgamma.double() - 0.25, ref.fn.norm.gamma.grad.reshape(-1)),
        "dtable": rel(dtable.double(), rp.relative_attention_bias.weight.grad),
        "dWqkv": rel(dwq.double() - 0.5, ref.fn.fn.fn.to_qkv.weight.grad),
        "dWout": rel(dwo, ref.fn.fn.fn.to_out.weight.grad),
        # O from the backward's P vs the forward's O (both bf16 P . V): rounding-level only
        "O_bwd_vs_fwd": rel(ob.double(), o.double()),
    }
    print(f"tblock fold/dw C=64 F={Fr} B={B} {H}x{W}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v < 3e-2, (k, v)
    assert errs["O_bwd_vs_fwd"] < 1e-2


@pytest.mark.parametrize("H,W", [(8, 8), (12, 20), (37, 29), (48, 96)])
def test_sla_fold_forward_and_dw_backward(dev, H, W):
    """the level-0 SLA training path at C = 64: slaf_fwd with LN gamma folded into W_qkv (pack_scaled, unit
    gamma) + cesm_slaf_bwd_dw (head-parallel backward, in-kernel dW_qkv / dgamma, no dqkv / xn
    intermediates) vs float64 autograd through the reference block (video_net.py:313-347); pixel counts
    that leave partial 48-pixel groups"""
    C = 64
    torch.manual_seed(15)
    B, Fr = 2, 3
    res = _sla_block(C, dev)
    sla = res.fn.fn
    x = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    g = q(torch.randn(B, C, Fr, H, W), torch.bfloat16)
    xd = to_cl(x).to(dev, torch.bfloat16)
    gd = to_cl(g).to(dev, torch.bfloat16)
    wqkv = sla.to_qkv.weight.detach().reshape(768, C).contiguous()
    wout = sla.to_out.weight.detach().reshape(C, 256)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    gamma = res.fn.norm.gamma.detach().reshape(-1).contiguous()
    ones = torch.ones(C, device=dev)
    wq_fold = K.pack_scaled(wqkv, gamma)
    assert torch.equal(wq_fold.float().cpu(), (wqkv * gamma).to(torch.bfloat16).float().cpu())
    assert torch.equal(K.pack_scaled(wqkv, gamma, trans=True), wq_fold.t().contiguous())
    y, st = K.slaf_fwd(xd, ones, wq_fold, wo, sla.to_out.bias.detach(), sla.scale, save_o=True)
    dgamma = torch.full((C,), 0.25, device=dev)
    dwq = torch.full((768, C), 0.5, device=dev)
    assert K.slaf_bwd_dw_supported(B * Fr, H * W, C)
    dx = K.slaf_bwd_dw(xd, gd, ones, wq_fold, wqkv, gamma, wo_t, st, dwq, dgamma, sla.scale)
    torch.cuda.synchronize()
    o = st[4]
    dwo = gd.reshape(-1, C).double().t() @ o.reshape(-1, 256).double()
    ref = _sla_block_ref(res, C)
    ref.fn.fn.to_qkv.weight.data.copy_(sla.to_qkv.weight.detach().cpu().double())  # fp32 master (folded in bf16)
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    (yr * g.double()).sum().backward()
    # the training path's to_out gradients: in the dctx pass from the recomputed q~ and the saved context
    # (the forward then writes no O); accumulated onto 0.5 / 0.25
    _, st_no = K.slaf_fwd(xd, ones, wq_fold, wo, sla.to_out.bias.detach(), sla.scale, save_o=False)
    assert st_no[4] is None
    dwo_k = torch.full((C, 256), 0.5, device=dev)
    dbo_k = torch.full((C,), 0.25, device=dev)
    dx2 = K.slaf_bwd_dw(xd, gd, ones, wq_fold, wqkv, gamma, wo_t, st_no, torch.zeros(768, C, device=dev),
                        torch.zeros(C, device=dev), sla.scale, dwout=dwo_k, dbout=dbo_k)
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx)
    errs = {
        "y": rel(from_cl(y, B), yr.detach()),
        "dx": rel(from_cl(dx, B), xr.grad),
        "dgamma": rel(dgamma.double() - 0.25, ref.fn.norm.gamma.grad.reshape(-1)),
        "dWqkv": rel(dwq.double() - 0.5, ref.fn.fn.to_qkv.weight.grad.reshape(768, C)),
        "dWout": rel(dwo, ref.fn.fn.to_out.weight.grad.reshape(C, 256)),
        "dWout_inkernel": rel(dwo_k.double() - 0.5, ref.fn.fn.to_out.weight.grad.reshape(C, 256)),
        "dbout_inkernel": rel(dbo_k.double() - 0.25, ref.fn.fn.to_out.bias.grad.reshape(-1)),
    }
    print(f"sla fold/dw HxW={H}x{W}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v < 3e-2, (k, v)


@pytest.mark.parametrize("F,HW,B", [(120, 77, 2), (33, 300, 1), (17, 40, 3)])
def test_tflash_pixel_major_matches_frame_major(dev, F, HW, B):
    """the long-window attention core with pixel-major qkv rows ([B][HW][F], the layout the F > 16 path's LN / to_qkv
    produce) gives the frame-major core's output bit for bit and the same gradients (dq / dk / dv in the same
    pixel-major order; the dq kernels differ below 32768 pixels -- D from dO . O vs sum P dP -- hence a tolerance)"""
    torch.manual_seed(F + HW)
    scale = 32 ** -0.5
    freqs = 1.0 / (10000 ** (torch.arange(0, 32, 2).float() / 32))
    bias = K.relpos_fwd(torch.randn(32, 8).to(dev), F)
    rot = K.rope_table(freqs.to(dev), F)
    qkv = torch.randn(B * F * HW, 768, device=dev).to(torch.bfloat16)
    to_pm = lambda t: t.view(B, F, HW, -1).transpose(1, 2).reshape(B * F * HW, -1).contiguous()  # noqa: E731
    from_pm = lambda t: t.view(B, HW, F, -1).transpose(1, 2).reshape(B * F * HW, -1)  # noqa: E731
    out, lse = K.tattn_fwd(qkv, bias, rot, B, F, HW, scale)
    out_pm, lse_pm = K.tattn_fwd(to_pm(qkv), bias, rot, B, F, HW, scale, pixel_major=True)
    assert torch.equal(out, out_pm) and torch.equal(lse, lse_pm)
    g = torch.randn(B * F * HW, 256, device=dev).to(torch.bfloat16)
    dt, dt_pm = torch.zeros(32, 8, device=dev), torch.zeros(32, 8, device=dev)
    dqkv = K.tattn_bwd(qkv, out, g, lse, bias, rot, dt, B, F, HW, scale)
    dqkv_pm = K.tattn_bwd(to_pm(qkv), out_pm, g, lse_pm, bias, rot, dt_pm, B, F, HW, scale, pixel_major=True)
    torch.cuda.synchronize()
    assert rel(from_pm(dqkv_pm).float(), dqkv.float()) < 1e-2
    assert rel(dt_pm, dt) < 1e-3


# ------------------------------------------------------------------ non-finite propagation (-fno-honor-nans)
# The attention sources are built without NaN semantics (cesm_emulator_amd/build.py NO_NANS): the compiler may treat
# fmaxf / comparisons as NaN-free.  The hardware arithmetic still propagates a NaN, and these tests pin that a NaN
# entering the attention kernels leaves them non-finite -- crossing frames (temporal) and pixels (spatial) through the
# attention mixing itself, not only along the residual -- so the reference's guard (train.py:860-861: a non-finite
# loss skips the step) still sees it.
def _nan_at(x, idx):
    x = x.clone()
    x[idx] = float("nan")
    return x


def test_nan_crosses_frames_in_fused_temporal_block(dev):
    """cesm_tblock_fwd_fold / cesm_tblock_bwd_dw (C = 64, F = 12): a NaN in x at one voxel makes y non-finite at every
    frame of that pixel (the softmax over frames mixes it in) and nowhere else; a NaN in dy at one voxel makes dx
    non-finite at every frame of that pixel and the weight gradient non-finite"""
    C, B, Fr, H, W = 64, 2, 12, 8, 12
    torch.manual_seed(5)
    rot_mod = VN.RotaryEmbedding(32)
    res_mod = VN.Residual(VN.PreNorm(C, VN.EinopsToAndFrom(VN.Attention(C, 8, 32, rot_mod)))).to(dev)
    attn = res_mod.fn.fn.fn
    rc = make_rc(B, Fr, torch.bfloat16)
    rc.bias = K.relpos_fwd(torch.randn(32, 8).to(dev), Fr)
    rc.rot = K.rope_table(rot_mod.freqs.to(dev), Fr)
    wqkv = attn.to_qkv.weight.detach().contiguous()
    wout = attn.to_out.weight.detach()
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    gamma = res_mod.fn.norm.gamma.detach().reshape(-1).contiguous()
    x = torch.randn(B, C, Fr, H, W)
    g = torch.randn(B, C, Fr, H, W)
    b0, f0, h0, w0 = 1, 4, 3, 7
    xd = to_cl(_nan_at(x, (b0, slice(None), f0, h0, w0))).to(dev, torch.bfloat16)
    y, mr, lse, _ = K.tblock_fwd_fold(xd, gamma, wqkv, wo, rc.bias, rc.rot, B, Fr, attn.scale)
    torch.cuda.synchronize()
    fin = torch.isfinite(from_cl(y, B).float().cpu()).all(dim=1)          # [B, F, H, W]
    assert not fin[b0, :, h0, w0].any(), "a NaN at one frame must reach every frame of its pixel"
    fin[b0, :, h0, w0] = True
    assert fin.all(), "the NaN leaked to other pixels"
    # backward: clean forward, NaN in dy at one voxel
    xd = to_cl(x).to(dev, torch.bfloat16)
    y, mr, lse, _ = K.tblock_fwd_fold(xd, gamma, wqkv, wo, rc.bias, rc.rot, B, Fr, attn.scale)
    gd = to_cl(_nan_at(g, (b0, slice(None), f0, h0, w0))).to(dev, torch.bfloat16)
    dgamma = torch.zeros(C, device=dev)
    dtable = torch.zeros(32, 8, device=dev)
    dwq = torch.zeros(768, C, device=dev)
    dx = K.tblock_bwd_dw(xd, gd, mr, lse, wqkv, gamma, wo_t, rc.bias, rc.rot, dwq, dgamma, dtable, B, Fr, attn.scale)
    torch.cuda.synchronize()
    fin = torch.isfinite(from_cl(dx, B).float().cpu()).all(dim=1)
    assert not fin[b0, :, h0, w0].any()
    fin[b0, :, h0, w0] = True
    assert fin.all()
    assert not torch.isfinite(dwq).all() and not torch.isfinite(dgamma).all()


def test_nan_crosses_pixels_in_fused_sla_block(dev):
    """cesm_slaf_fwd / cesm_slaf_bwd_dw (C = 64): a NaN in x at one pixel of a frame makes y non-finite over that whole
    frame (the context sums every pixel's k v^T) and in no other frame; a NaN in dy at one pixel does the same to dx"""
    C, B, Fr, H, W = 64, 1, 3, 12, 20
    torch.manual_seed(6)
    res = _sla_block(C, dev)
    sla = res.fn.fn
    wqkv = sla.to_qkv.weight.detach().reshape(768, C).contiguous()
    wout = sla.to_out.weight.detach().reshape(C, 256)
    wo = K.conv_pack(wout, torch.bfloat16, C, 256, 1, 1, 0, 0)
    wo_t = K.conv_pack(wout, torch.bfloat16, 256, C, 1, 1, 1, 1)
    gamma = res.fn.norm.gamma.detach().reshape(-1).contiguous()
    ones = torch.ones(C, device=dev)
    wq_fold = K.pack_scaled(wqkv, gamma)
    x = torch.randn(B, C, Fr, H, W)
    g = torch.randn(B, C, Fr, H, W)
    f0, h0, w0 = 1, 5, 11
    xd = to_cl(_nan_at(x, (0, slice(None), f0, h0, w0))).to(dev, torch.bfloat16)
    y, st = K.slaf_fwd(xd, ones, wq_fold, wo, sla.to_out.bias.detach(), sla.scale)
    torch.cuda.synchronize()
    fin = torch.isfinite(from_cl(y, B).float().cpu()).all(dim=1)[0]       # [F, H, W]
    assert not fin[f0].any(), "a NaN at one pixel must reach every pixel of its frame"
    assert fin[[f for f in range(Fr) if f != f0]].all()
    xd = to_cl(x).to(dev, torch.bfloat16)
    y, st = K.slaf_fwd(xd, ones, wq_fold, wo, sla.to_out.bias.detach(), sla.scale)
    gd = to_cl(_nan_at(g, (0, slice(None), f0, h0, w0))).to(dev, torch.bfloat16)
    dwq = torch.zeros(768, C, device=dev)
    dgamma = torch.zeros(C, device=dev)
    dx = K.slaf_bwd_dw(xd, gd, ones, wq_fold, wqkv, gamma, wo_t, st, dwq, dgamma, sla.scale)
    torch.cuda.synchronize()
    fin = torch.isfinite(from_cl(dx, B).float().cpu()).all(dim=1)[0]
    assert not fin[f0].any()
    assert fin[[f for f in range(Fr) if f != f0]].all()
    assert not torch.isfinite(dwq).all()


@pytest.mark.parametrize("F", [12, 120])
def test_nan_crosses_frames_in_long_window_core(dev, F):
    """the MFMA long-window core (tflash, F <= 128): a NaN in one (pixel, frame) qkv row makes that pixel's output
    non-finite at every frame and leaves other pixels finite; a NaN in dout does the same to dqkv"""
    B, HW = 1, 37
    torch.manual_seed(F)
    scale = 32 ** -0.5
    freqs = 1.0 / (10000 ** (torch.arange(0, 32, 2).float() / 32))
    bias = K.relpos_fwd(torch.randn(32, 8).to(dev), F)
    rot = K.rope_table(freqs.to(dev), F)
    qkv = torch.randn(B * F * HW, 768)
    f0, p0 = F // 3, 17
    row = f0 * HW + p0                                                    # frame-major rows [B][F][HW]
    bad = qkv.clone()
    bad[row] = float("nan")
    out, lse = K.tattn_fwd(bad.to(dev, torch.bfloat16), bias, rot, B, F, HW, scale)
    torch.cuda.synchronize()
    fin = torch.isfinite(out.float().cpu()).all(dim=1).view(F, HW)
    assert not fin[:, p0].any()
    fin[:, p0] = True
    assert fin.all()
    qd = qkv.to(dev, torch.bfloat16)
    out, lse = K.tattn_fwd(qd, bias, rot, B, F, HW, scale)
    g = torch.randn(B * F * HW, 256)
    g[row] = float("nan")
    dqkv = K.tattn_bwd(qd, out, g.to(dev, torch.bfloat16), lse, bias, rot, torch.zeros(32, 8, device=dev),
                       B, F, HW, scale)
    torch.cuda.synchronize()
    fin = torch.isfinite(dqkv.float().cpu()).all(dim=1).view(F, HW)
    assert not fin[:, p0].any()
    fin[:, p0] = True
    assert fin.all()
