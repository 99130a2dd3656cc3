"""Drop-in replacement for the reference's model.py (UNet wrapper + DDPM Diffusion).

Same constructor kwargs (model.py:44-64), same `net.*` state_dict keys and the same 8 Diffusion
buffers (model.py:158-165), so train.py / inference.py / plot_*.py can import this module
unchanged.  Compute runs on libcesm_hip.so; there is no CPU path — call `.to("cuda")` first.

Precision: `UNet.compute_dtype` selects the activation storage type of the kernels —
torch.bfloat16 (default, training/throughput) or torch.float32 (parity mode: forward matches
the CPU fp32 reference within 1e-5 relative L2).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import kernels as K
from .video_net import UNetModel3D, net_apply


class UNet(nn.Module):
    """model.py:37-134."""

    def __init__(self, in_channels: int = 2, out_channels: int = 1, base_ch: int = 64, ch_mults=(1, 2, 4),
                 num_res_blocks: int = 2, time_dim: int = 256, groups: int = 8, dropout: float = 0.0,
                 attn_heads: int = 8, attn_dim_head: int = 32, use_sparse_linear_attn: bool = True,
                 use_mid_attn: bool = False, init_kernel_size: int = 7, use_checkpoint: bool = False,
                 use_temp_attn: bool = True, day_cond: bool = False, year_cond: bool = False,
                 cond_map: bool = True):
        super().__init__()
        self.net = UNetModel3D(n_vars=out_channels, model_dim=base_ch, dim_mults=tuple(ch_mults),
                               attn_heads=attn_heads, attn_dim_head=attn_dim_head,
                               use_sparse_linear_attn=use_sparse_linear_attn, use_mid_attn=use_mid_attn,
                               init_kernel_size=init_kernel_size, resnet_groups=groups,
                               use_checkpoint=use_checkpoint, use_temp_attn=use_temp_attn, day_cond=day_cond,
                               year_cond=year_cond, cond_map=cond_map)

    @property
    def compute_dtype(self):
        return self.net.compute_dtype

    @compute_dtype.setter
    def compute_dtype(self, dt):
        if dt not in (torch.float32, torch.bfloat16):
            raise ValueError("compute_dtype must be torch.float32 or torch.bfloat16")
        self.net.compute_dtype = dt
        self.net.invalidate_packed()

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
        Fx, Fc = x_t.shape[2], cond.shape[2]
        if Fx != Fc and not (Fx == 1 or Fc == 1):
            raise ValueError(f"Frame mismatch: x_t F={Fx}, cond F={Fc}")
        if x_t.shape[1] != 1 or cond.shape[1] != 1:
            raise ValueError("single-variable model: x_t and cond need 1 channel")
        if not x_t.is_cuda:
            raise RuntimeError("cesm_emulator_amd.UNet runs on the GPU only (move model and inputs to 'cuda')")
        if not torch.is_tensor(t):
            t = torch.tensor([t], dtype=torch.long, device=x_t.device)
        elif t.ndim == 0:
            t = t[None]
        t = t.to(device=x_t.device, dtype=torch.long).contiguous()
        if t.shape[0] == 1 and x_t.shape[0] > 1:
            t = t.expand(x_t.shape[0]).contiguous()
        # frame-broadcast of model.py:111-118 happens inside the stem kernel (stride-0 read)
        xt4 = x_t[:, 0].float().contiguous()
        c4 = cond[:, 0].float().contiguous()
        # the network's output is [B,1,F,H,W]; only frame F//2 is kept (model.py:124-130), so
        # the 1x1 head conv is evaluated on that frame only.
        return net_apply(self.net, xt4, c4, t)


class _MSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, noise):
        ctx.save_for_backward(pred, noise)
        return K.mse(pred, noise)

    @staticmethod
    def backward(ctx, g):
        pred, noise = ctx.saved_tensors
        return K.mse_bwd(pred, noise, g.reshape(1).contiguous()), None


class Diffusion(nn.Module):
    """model.py:141-208 — linear β schedule (1e-4 → 2e-2), ε-prediction MSE."""

    def __init__(self, model, img_channels=1, timesteps=1000, beta_schedule="linear"):
        super().__init__()
        self.model = model
        self.img_channels = img_channels
        self.T = timesteps
        if beta_schedule != "linear":
            raise ValueError("Only 'linear' beta_schedule implemented")
        betas = torch.linspace(1e-4, 2e-2, timesteps)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, dim=0)
        acp = torch.cat([torch.tensor([1.0]), ac[:-1]], dim=0)
        self.register_buffer("betas", betas)
        self.register_buffer("alphas", alphas)
        self.register_buffer("alphas_cumprod", ac)
        self.register_buffer("alphas_cumprod_prev", acp)
        self.register_buffer("sqrt_alphas_cumprod", torch.sqrt(ac))
        self.register_buffer("sqrt_one_minus_alphas_cumprod", torch.sqrt(1.0 - ac))
        self.register_buffer("sqrt_recip_alphas", torch.sqrt(1.0 / alphas))
        self.register_buffer("posterior_variance", betas * (1.0 - acp) / (1.0 - ac))
        # draws of t / eps in loss(): None = the default generator (as model.py:205-206); data-parallel
        # training gives every rank its own stream (train.rank_generator) so ranks do not draw identical
        # t / eps for their different samples
        self.generator = None

    def q_sample(self, x0, t, noise=None):
        if noise is None:
            noise = torch.randn_like(x0)
        xt = K.q_sample(x0.float().contiguous(), noise.float().contiguous(), t.long().contiguous(),
                        self.sqrt_alphas_cumprod, self.sqrt_one_minus_alphas_cumprod)
        return xt, noise

    def loss(self, x0, cond, t=None, noise=None):
        """model.py:203-208; optional t / noise make the draw reproducible for parity tests."""
        B = x0.size(0)
        g = self.generator
        if t is None:
            t = torch.randint(0, self.T, (B,), device=x0.device, generator=g).long()
        if noise is None:
            noise = torch.randn(x0.shape, device=x0.device, dtype=x0.dtype, generator=g)
        x_t, noise = self.q_sample(x0, t, noise)
        eps = self.model(x_t, cond, t)
        return _MSE.apply(eps, noise.float().contiguous())

    def _coefs(self):
        return self.sqrt_recip_alphas, self.betas, self.sqrt_one_minus_alphas_cumprod, self.posterior_variance

    @torch.no_grad()
    def p_sample(self, x_t, cond, t, noise=None):
        """model.py:168-183 (DDPM ancestral step): model evaluation + one fused update kernel."""
        with torch.inference_mode():
            x_t = x_t.float().contiguous()
            t = t.to(device=x_t.device, dtype=torch.long).contiguous()
            eps = self.model(x_t, cond, t).float().contiguous()
            if (t == 0).all():
                return K.ddpm_step(x_t, eps, None, t, *self._coefs())
            if noise is None:
                noise = torch.randn_like(x_t)
            return K.ddpm_step(x_t, eps, noise.float().contiguous(), t, *self._coefs())

    @torch.no_grad()
    def sample(self, cond, shape, device, use_graph=None, x_T=None, noise_seq=None):
        """model.py:186-194.  On the GPU every p_sample step is ONE replay of a captured HIP graph (the
        F=1 network forward + the fused update); the host only sets t and draws the step noise.  RNG use
        is the reference's: randn(shape) for x_T, then randn_like(x) for every step with t > 0, drawn
        outside the graph on the default generator, so the result equals the eager loop.  Test hooks:
        x_T (initial state) and noise_seq ([T, *shape], noise of step i = noise_seq[i], i = 0 for t = T-1)
        replace the draws.  use_graph=False (or CESM_SAMPLE_GRAPH=0) runs the eager loop."""
        with torch.inference_mode():
            B = shape[0]
            x = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float().clone()
            if use_graph is None:
                use_graph = os.environ.get("CESM_SAMPLE_GRAPH", "1") != "0"
            if not use_graph:
                for i, tt in enumerate(reversed(range(self.T))):
                    t_tensor = torch.full((B,), tt, device=device, dtype=torch.long)
                    nz = None if noise_seq is None or tt == 0 else noise_seq[i].to(device)
                    x = self.p_sample(x, cond, t_tensor, noise=nz)
                return x
            step = GraphSampleStep(self, cond, x)
            for i, tt in enumerate(reversed(range(self.T))):
                if tt == 0:
                    step.z.zero_()
                elif noise_seq is not None:
                    step.z.copy_(noise_seq[i])
                else:
                    step.z.normal_()
                step.run(tt)
            return step.x


class GraphSampleStep:
    """One DDPM sampling step (model eval + fused update, in place on a static x) captured as a HIP graph
    (torch.cuda.graph drives hipStreamBeginCapture; every kernel launches on the capturing stream).
    Static inputs: x [B,1,H,W] fp32 (updated in place), cond, t [B] int64, z (step noise; zero at t=0,
    where posterior_variance[0] = 0 makes the noise term vanish as in the reference's t=0 branch)."""

    def __init__(self, diffusion, cond, x):
        self.d = diffusion
        self.x = x.float().contiguous()
        self.cond = cond.float().contiguous()
        self.t = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        self.z = torch.zeros_like(self.x)
        x0 = self.x.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: weight packs, lazily built tables, allocator pools
            for _ in range(2):
                self._step()
        torch.cuda.current_stream().wait_stream(side)
        self.x.copy_(x0)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._step()

    def _step(self):
        eps = self.d.model(self.x, self.cond, self.t).float().contiguous()
        K.ddpm_step(self.x, eps, self.z, self.t, *self.d._coefs(), out=self.x)

    def run(self, tt):
        self.t.fill_(tt)
        self.graph.replay()
