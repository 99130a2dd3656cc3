"""CPU fp32 restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle (and the `cpu_baseline` leg of bench.py).  Only
`tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline may import it; the
product package `cesm_emulator_amd` never does.

It restates, op for op in plain PyTorch-CPU fp32, the reference's
  * video_net.py  (UNetModel3D and the blocks it instantiates)
  * rotary_embedding.py (the subset video_net uses: lang freqs, rotate_queries_or_keys)
  * model.py      (UNet wrapper, Diffusion schedule / q_sample / loss / p_sample / sample)
  * train.py:868-880 fp32 step: loss → backward → clip_grad_norm_(1.0) → AdamW
with the module tree laid out so `state_dict()` keys equal the reference's.

Parity status: the reference ships no tests, fixtures or golden vectors and importing
it was denied by the environment, so this restatement is pinned
by the hand-derived known-answer tests of SURVEY.md §8(c) C5 (tests/test_oracle.py)
and the parameter counts of §8(d) D4 — "parity pinned by known answers only".
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------- helpers
class Identity(nn.Module):
    def forward(self, x, *args, **kwargs):
        return x


def Downsample(dim):  # video_net.py:61-62
    return nn.Conv3d(dim, dim, (1, 4, 4), (1, 2, 2), (0, 1, 1))


def Upsample(dim):  # video_net.py:65-66
    return nn.ConvTranspose3d(dim, dim, (1, 4, 4), (1, 2, 2), (0, 1, 1))


class Residual(nn.Module):  # video_net.py:69-75
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, *args, **kwargs):
        return self.fn(x, *args, **kwargs) + x


class LayerNorm(nn.Module):  # video_net.py:78-87 — channel LN, biased var, gamma only
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(1, dim, 1, 1, 1))

    def forward(self, x):
        mu = x.mean(dim=1, keepdim=True)
        var = ((x - mu) ** 2).mean(dim=1, keepdim=True)
        return (x - mu) / torch.sqrt(var + self.eps) * self.gamma


class PreNorm(nn.Module):  # video_net.py:90-98
    def __init__(self, dim, fn):
        super().__init__()
        self.fn = fn
        self.norm = LayerNorm(dim)

    def forward(self, x, **kwargs):
        return self.fn(self.norm(x), **kwargs)


class SinusoidalPosEmb(nn.Module):  # video_net.py:101-113
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, x):
        half = self.dim // 2
        step = math.log(10000) / (half - 1)
        freqs = torch.exp(torch.arange(half, device=x.device) * -step)
        arg = x[:, None] * freqs[None, :]
        return torch.cat((arg.sin(), arg.cos()), dim=-1)


# --------------------------------------------------------------------------- rotary
class RotaryEmbedding(nn.Module):
    """rotary_embedding.py:62-134 (freqs_for='lang'), :143-163, :254-283."""

    def __init__(self, dim, theta=10000):
        super().__init__()
        freqs = 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))
        self.freqs = nn.Parameter(freqs, requires_grad=False)

    def angles(self, seq_len, dtype):
        # get_seq_pos in the input dtype (:143-144), then cast to freqs dtype (:277)
        pos = torch.arange(seq_len, dtype=dtype).to(self.freqs.dtype)
        ang = pos[:, None] * self.freqs[None, :]
        return ang.repeat_interleave(2, dim=-1)  # '... n -> ... (n r)', r=2 (:278)

    @staticmethod
    def rotate_half(x):  # :29-33 — pairs (x[2i], x[2i+1]) -> (-x[2i+1], x[2i])
        x = x.unflatten(-1, (-1, 2))
        x1, x2 = x.unbind(-1)
        return torch.stack((-x2, x1), dim=-1).flatten(-2)

    def rotate_queries_or_keys(self, t):  # seq dim = -2 (default_seq_dim)
        ang = self.angles(t.shape[-2], t.dtype)
        return t * ang.cos() + self.rotate_half(t) * ang.sin()  # apply_rotary_emb :35-48


# --------------------------------------------------------------------------- blocks
class Block(nn.Module):  # video_net.py:212-227
    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.proj = nn.Conv3d(dim, dim_out, (1, 3, 3), padding=(0, 1, 1))
        self.norm = nn.GroupNorm(groups, dim_out)

    def forward(self, x, scale_shift=None):
        x = self.norm(self.proj(x))
        if scale_shift is not None:
            scale, shift = scale_shift
            x = x * (scale + 1) + shift
        return F.silu(x)


class ResnetBlock(nn.Module):  # video_net.py:230-265
    def __init__(self, dim, dim_out, *, time_emb_dim=None, groups=8):
        super().__init__()
        self.mlp = (nn.Sequential(nn.SiLU(), nn.Linear(time_emb_dim, dim_out * 2))
                    if time_emb_dim is not None else None)
        self.block1 = Block(dim, dim_out, groups=groups)
        self.block2 = Block(dim_out, dim_out, groups=groups)
        self.res_conv = nn.Conv3d(dim, dim_out, 1) if dim != dim_out else nn.Identity()

    def forward(self, x, time_emb=None):
        ss = None
        if self.mlp is not None:
            te = self.mlp(time_emb)[:, :, None, None, None]
            ss = te.chunk(2, dim=1)
        h = self.block1(x, scale_shift=ss)
        h = self.block2(h)
        return h + self.res_conv(x)


class RelativePositionBias(nn.Module):  # video_net.py:268-310
    def __init__(self, heads=8, num_buckets=32, max_distance=128):
        super().__init__()
        self.num_buckets = num_buckets
        self.max_distance = max_distance
        self.relative_attention_bias = nn.Embedding(num_buckets, heads)

    @staticmethod
    def bucket(rel, num_buckets=32, max_distance=128):
        n = -rel
        nb = num_buckets // 2
        ret = (n < 0).long() * nb
        n = n.abs()
        max_exact = nb // 2
        small = n < max_exact
        large = max_exact + (torch.log(n.float() / max_exact) / math.log(max_distance / max_exact)
                             * (nb - max_exact)).long()
        large = torch.minimum(large, torch.full_like(large, nb - 1))
        return ret + torch.where(small, n, large)

    def forward(self, n, device=None):
        pos = torch.arange(n, dtype=torch.long)
        rel = pos[None, :] - pos[:, None]  # k_pos - q_pos  (j - i)
        b = self.bucket(rel, self.num_buckets, self.max_distance)
        return self.relative_attention_bias(b).permute(2, 0, 1)  # 'i j h -> h i j'


class SpatialLinearAttention(nn.Module):  # video_net.py:313-347
    def __init__(self, dim, heads=4, dim_head=32):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        hidden = dim_head * heads
        self.to_qkv = nn.Conv2d(dim, hidden * 3, 1, bias=False)
        self.to_out = nn.Conv2d(hidden, dim, 1)

    def forward(self, x):
        b, c, f, h, w = x.shape
        x = x.permute(0, 2, 1, 3, 4).reshape(b * f, c, h, w)
        q, k, v = self.to_qkv(x).chunk(3, dim=1)
        q, k, v = (t.reshape(b * f, self.heads, -1, h * w) for t in (q, k, v))  # b (h c) x y -> b h c (xy)
        q = q.softmax(dim=-2)
        k = k.softmax(dim=-1)
        q = q * self.scale
        ctx = torch.einsum("bhdn,bhen->bhde", k, v)
        out = torch.einsum("bhde,bhdn->bhen", ctx, q)
        out = self.to_out(out.reshape(b * f, -1, h, w))
        return out.reshape(b, f, c, h, w).permute(0, 2, 1, 3, 4)


class Attention(nn.Module):  # video_net.py:368-454 (focus mask inert: prob 0)
    def __init__(self, dim, heads=4, dim_head=32, rotary_emb=None):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        hidden = dim_head * heads
        self.rotary_emb = rotary_emb
        self.to_qkv = nn.Linear(dim, hidden * 3, bias=False)
        self.to_out = nn.Linear(hidden, dim, bias=False)

    def forward(self, x, pos_bias=None, focus_present_mask=None):
        q, k, v = self.to_qkv(x).chunk(3, dim=-1)
        q, k, v = (t.unflatten(-1, (self.heads, -1)).transpose(-2, -3) for t in (q, k, v))
        q = q * self.scale
        if self.rotary_emb is not None:
            q = self.rotary_emb.rotate_queries_or_keys(q)
            k = self.rotary_emb.rotate_queries_or_keys(k)
        sim = torch.einsum("...hid,...hjd->...hij", q, k)
        if pos_bias is not None:
            sim = sim + pos_bias
        sim = sim - sim.amax(dim=-1, keepdim=True).detach()
        attn = sim.softmax(dim=-1)
        out = torch.einsum("...hij,...hjd->...hid", attn, v)
        out = out.transpose(-2, -3).flatten(-2)
        return self.to_out(out)


class EinopsToAndFrom(nn.Module):
    """video_net.py:350-365 with the only pattern used: 'b c f h w' <-> 'b (h w) f c'."""

    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, **kwargs):
        b, c, f, h, w = x.shape
        y = x.permute(0, 3, 4, 2, 1).reshape(b, h * w, f, c)
        y = self.fn(y, **kwargs)
        return y.reshape(b, h, w, f, c).permute(0, 4, 3, 1, 2)


# --------------------------------------------------------------------------- network
class UNetModel3D(nn.Module):
    """video_net.py:562-871, with the flags model.UNet passes (no day/year cond,
    use_temp_attn=True, cond_map=True).  Module construction order follows the
    reference so a fixed torch seed yields the reference's initial weights."""

    def __init__(self, n_vars, model_dim, dim_mults=(1, 2, 4, 8), attn_heads=8, attn_dim_head=32,
                 use_sparse_linear_attn=True, use_mid_attn=False, init_kernel_size=7,
                 resnet_groups=8):
        super().__init__()
        in_ch = 2 * n_vars
        pad = init_kernel_size // 2
        self.input_conv = nn.Conv3d(in_ch, model_dim, (1, init_kernel_size, init_kernel_size),
                                    padding=(0, pad, pad))
        rotary = RotaryEmbedding(min(32, attn_dim_head))
        # the reference builds RelativePositionBias twice (:605, :630); keep the RNG draw
        self.time_rel_pos_bias = RelativePositionBias(heads=attn_heads, max_distance=32)
        self.time_rel_pos_bias = RelativePositionBias(heads=attn_heads, max_distance=32)

        def tattn(dim):
            return EinopsToAndFrom(Attention(dim, heads=attn_heads, dim_head=attn_dim_head,
                                             rotary_emb=rotary))

        self.input_temp_op = Residual(PreNorm(model_dim, tattn(model_dim)))
        dims = [model_dim, *[int(model_dim * m) for m in dim_mults]]
        in_out = list(zip(dims[:-1], dims[1:]))
        time_dim = model_dim * 4
        self.time_mlp = nn.Sequential(SinusoidalPosEmb(model_dim), nn.Linear(model_dim, time_dim),
                                      nn.SiLU(), nn.Linear(time_dim, time_dim))
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
        self.mid_spatial_attn = nn.Identity()  # use_mid_attn=False (model.py:57)
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

    def forward(self, x, timesteps, cond_map=None):
        bias = self.time_rel_pos_bias(x.shape[2])
        if cond_map is not None:
            x = torch.cat([x, cond_map], dim=1)
        x = self.input_conv(x)
        x = self.input_temp_op(x, pos_bias=bias)
        r = x.clone()
        t = self.time_mlp(timesteps)
        hs = []
        for b1, b2, sa, ta, down in self.downs:
            x = b1(x, t)
            x = b2(x, t)
            x = sa(x)
            x = ta(x, pos_bias=bias)
            hs.append(x)
            x = down(x)
        x = self.mid_block1(x, t)
        x = self.mid_spatial_attn(x)
        x = self.mid_temporal_attn(x, pos_bias=bias)
        x = self.mid_block2(x, t)
        for b1, b2, sa, ta, up in self.ups:
            x = torch.cat((x, hs.pop()), dim=1)
            x = b1(x, t)
            x = b2(x, t)
            x = sa(x)
            x = ta(x, pos_bias=bias)
            x = up(x)
        x = torch.cat((x, r), dim=1)
        return self.out_conv(x)


class UNet(nn.Module):
    """model.py:37-134 — same constructor kwargs, same `net.*` state_dict keys."""

    def __init__(self, in_channels=2, out_channels=1, base_ch=64, ch_mults=(1, 2, 4),
                 num_res_blocks=2, time_dim=256, groups=8, dropout=0.0, attn_heads=8,
                 attn_dim_head=32, use_sparse_linear_attn=True, use_mid_attn=False,
                 init_kernel_size=7, use_checkpoint=False, use_temp_attn=True,
                 day_cond=False, year_cond=False, cond_map=True):
        super().__init__()
        self.net = UNetModel3D(n_vars=out_channels, model_dim=base_ch, dim_mults=tuple(ch_mults),
                               attn_heads=attn_heads, attn_dim_head=attn_dim_head,
                               use_sparse_linear_attn=use_sparse_linear_attn,
                               use_mid_attn=use_mid_attn, init_kernel_size=init_kernel_size,
                               resnet_groups=groups)

    def forward(self, x_t, cond, t):
        if x_t.ndim == 4:
            x_t = x_t.unsqueeze(2)
        elif x_t.ndim != 5:
            raise ValueError(f"x_t must be 4D or 5D, got {x_t.ndim}D")
        if cond is None:
            raise ValueError("cond must be provided")
        if cond.ndim == 4:
            cond = cond.unsqueeze(2)
        elif cond.ndim != 5:
            raise ValueError(f"cond must be 4D or 5D, got {cond.ndim}D")
        fx, fc = x_t.shape[2], cond.shape[2]
        if fx != fc:
            if fx == 1:
                x_t = x_t.expand(-1, -1, fc, -1, -1)
            elif fc == 1:
                cond = cond.expand(-1, -1, fx, -1, -1)
            else:
                raise ValueError(f"Frame mismatch: x_t F={fx}, cond F={fc}")
        if not torch.is_tensor(t):
            t = torch.tensor([t], dtype=torch.long)
        elif t.ndim == 0:
            t = t[None]
        out = self.net(x_t, t, cond_map=cond)
        return out[:, :, out.shape[2] // 2] if out.shape[2] > 1 else out.squeeze(2)


class Diffusion(nn.Module):
    """model.py:141-208 (linear β schedule, ε-prediction MSE)."""

    def __init__(self, model, img_channels=1, timesteps=1000, beta_schedule="linear"):
        super().__init__()
        if beta_schedule != "linear":
            raise ValueError("Only 'linear' beta_schedule implemented")
        self.model = model
        self.img_channels = img_channels
        self.T = timesteps
        betas = torch.linspace(1e-4, 2e-2, timesteps)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, dim=0)
        acp = torch.cat([torch.tensor([1.0]), ac[:-1]])
        for name, val in (("betas", betas), ("alphas", alphas), ("alphas_cumprod", ac),
                          ("alphas_cumprod_prev", acp), ("sqrt_alphas_cumprod", ac.sqrt()),
                          ("sqrt_one_minus_alphas_cumprod", (1.0 - ac).sqrt()),
                          ("sqrt_recip_alphas", (1.0 / alphas).sqrt()),
                          ("posterior_variance", betas * (1.0 - acp) / (1.0 - ac))):
            self.register_buffer(name, val)

    def q_sample(self, x0, t, noise=None):
        if noise is None:
            noise = torch.randn_like(x0)
        a = self.sqrt_alphas_cumprod[t].view(-1, 1, 1, 1)
        s = self.sqrt_one_minus_alphas_cumprod[t].view(-1, 1, 1, 1)
        return a * x0 + s * noise, noise

    def loss(self, x0, cond, t=None, noise=None):
        if t is None:
            t = torch.randint(0, self.T, (x0.size(0),), device=x0.device).long()
        x_t, noise = self.q_sample(x0, t, noise)
        return F.mse_loss(self.model(x_t, cond, t), noise)

    @torch.no_grad()
    def p_sample(self, x_t, cond, t, noise=None):
        b = self.betas[t].view(-1, 1, 1, 1)
        s1 = self.sqrt_one_minus_alphas_cumprod[t].view(-1, 1, 1, 1)
        r = self.sqrt_recip_alphas[t].view(-1, 1, 1, 1)
        eps = self.model(x_t, cond, t)
        mean = r * (x_t - b / s1 * eps)
        if (t == 0).all():
            return mean
        if noise is None:
            noise = torch.randn_like(x_t)
        return mean + torch.sqrt(self.posterior_variance[t].view(-1, 1, 1, 1)) * noise

    @torch.no_grad()
    def sample(self, cond, shape, device, x_T=None, noise_seq=None):
        """model.py:186-194; x_T / noise_seq ([T, *shape], step i <-> t = T-1-i) replace the draws."""
        B = shape[0]
        x = torch.randn(shape, device=device) if x_T is None else x_T.clone()
        for i, tt in enumerate(reversed(range(self.T))):
            t = torch.full((B,), tt, device=device, dtype=torch.long)
            x = self.p_sample(x, cond, t, None if noise_seq is None or tt == 0 else noise_seq[i])
        return x


def train_step(diffusion, optimizer, x0, cond, t=None, noise=None, max_grad_norm=1.0):
    """train.py:868-880 (fp32 branch): zero_grad → loss → isfinite → backward → clip → step."""
    optimizer.zero_grad(set_to_none=True)
    loss = diffusion.loss(x0, cond, t=t, noise=noise)
    if not torch.isfinite(loss):
        raise RuntimeError(f"Non-finite loss: {loss.item()}")
    loss.backward()
    if max_grad_norm is not None and max_grad_norm > 0:
        torch.nn.utils.clip_grad_norm_(diffusion.parameters(), max_grad_norm)
    optimizer.step()
    return loss.detach()


def make_optimizer(diffusion, lr=2e-4, betas=(0.9, 0.999), weight_decay=1e-4):
    """train.py:1077-1083."""
    return torch.optim.AdamW(diffusion.parameters(), lr=lr, betas=betas, weight_decay=weight_decay)


def config_unet_kwargs(cfg_unet):
    """train.py:669-680 build_model_from_config kwargs."""
    return dict(in_channels=cfg_unet.get("in_channels", 2), out_channels=cfg_unet.get("out_channels", 1),
                base_ch=cfg_unet.get("base_ch", 64), ch_mults=tuple(cfg_unet.get("ch_mults", (1, 2, 4))),
                num_res_blocks=cfg_unet.get("num_res_blocks", 2), time_dim=cfg_unet.get("time_dim", 256),
                groups=cfg_unet.get("groups", 8), use_checkpoint=cfg_unet.get("use_checkpoint", True),
                dropout=cfg_unet.get("dropout", 0.0))
