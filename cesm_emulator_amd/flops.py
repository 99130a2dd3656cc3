"""Algorithmic MAC count of one UNet forward (video_net.py:562-871), derived from the module shapes.

Counts every multiply-accumulate of the dense contractions: convs (stem, 3x3, 1x1 res, 4x4 down,
4x4 transposed up), attention projections (to_qkv / to_out), the temporal-attention core (q.k and
attn.v: 2*F*32 per query per head) and the spatial-linear-attention core (context k.v^T and
context^T.q: 2*32*32 per position per head).  Training FLOPs/sample = 3 * 2 * forward MACs
(fwd + dgrad + wgrad), the convention of SURVEY.md §8(d) D4.  The head conv is counted on every
frame although only frame F//2 is evaluated (64 MAC/voxel, < 0.01 %).
"""
from __future__ import annotations

import torch.nn as nn


def unet_forward_macs(net, F, H, W):
    """net: cesm_emulator_amd.video_net.UNetModel3D (or the oracle's); per-sample MACs."""
    macs = 0
    h, w = H, W

    def conv(mod, hh, ww):
        wt = mod.weight
        if isinstance(mod, nn.ConvTranspose3d):
            return F * hh * ww * wt.shape[0] * wt.shape[1] * wt.shape[-1] * wt.shape[-2]
        k = wt.shape[-1] * wt.shape[-2] if wt.dim() >= 4 else 1
        s = mod.stride[-1] if hasattr(mod, "stride") else 1
        return F * (hh // s) * (ww // s) * wt.shape[0] * wt.shape[1] * k

    def resnet(rb, hh, ww):
        m = conv(rb.block1.proj, hh, ww) + conv(rb.block2.proj, hh, ww)
        if not isinstance(rb.res_conv, nn.Identity):
            m += conv(rb.res_conv, hh, ww)
        if rb.mlp is not None:
            lin = rb.mlp[1]
            m += lin.in_features * lin.out_features
        return m

    def tattn(res_mod, hh, ww):
        a = res_mod.fn.fn.fn
        v = F * hh * ww
        d = a.to_qkv.in_features
        return v * (768 * d + 256 * d) + v * 8 * 2 * F * 32

    def sla(res_mod, hh, ww):
        s = res_mod.fn.fn
        v = F * hh * ww
        d = s.to_qkv.weight.shape[1]
        return v * (768 * d + 256 * d) + v * 8 * 2 * 32 * 32

    macs += conv(net.input_conv, h, w)
    macs += tattn(net.input_temp_op, h, w)
    lins = [net.time_mlp[1], net.time_mlp[3]]
    macs += sum(l.in_features * l.out_features for l in lins)
    for b1, b2, sa, ta, down in net.downs:
        macs += resnet(b1, h, w) + resnet(b2, h, w)
        if not isinstance(sa, nn.Identity):
            macs += sla(sa, h, w)
        macs += tattn(ta, h, w)
        if not isinstance(down, nn.Identity):
            macs += conv(down, h, w)
            h, w = h // 2, w // 2
    macs += resnet(net.mid_block1, h, w) + tattn(net.mid_temporal_attn, h, w) + resnet(net.mid_block2, h, w)
    for b1, b2, sa, ta, up in net.ups:
        macs += resnet(b1, h, w) + resnet(b2, h, w)
        if not isinstance(sa, nn.Identity):
            macs += sla(sa, h, w)
        macs += tattn(ta, h, w)
        if not isinstance(up, nn.Identity):
            macs += conv(up, h, w)
            h, w = h * 2, w * 2
    macs += resnet(net.out_conv[0], h, w)
    macs += F * h * w * net.out_conv[1].weight.shape[1]
    return macs


def train_flops_per_sample(net, F, H, W):
    return 6 * unet_forward_macs(net, F, H, W)
