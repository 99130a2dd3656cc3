"""Fused AdamW + global-norm gradient clipping over one flat fp32 parameter buffer.

Replaces `torch.optim.AdamW(diffusion.parameters(), lr, betas, weight_decay)` (train.py:1077-1083)
and `torch.nn.utils.clip_grad_norm_(diffusion.parameters(), max_grad_norm)` (train.py:865).

At construction all trainable parameters are moved into one contiguous fp32 buffer (each
`param.data` becomes a view into it) and their `.grad` into a second one.  That makes the whole
optimizer step two kernel launches (norm reduction + fused AdamW; no host sync — the clip
coefficient and the finite-check stay on the device) and lets the data-parallel all-reduce work
on a handful of large contiguous buckets.  Math follows torch/optim/adam.py:417-547 (decoupled
weight decay, bias corrections, eps outside the sqrt) and torch/nn/utils/clip_grad.py:165-180.
"""
from __future__ import annotations

import torch
from . import kernels as K
from .video_net import bump_param_epoch


class FlatParams:
    """Packs parameters (and their grads) into contiguous fp32 buffers."""

    def __init__(self, params):
        seen, plist = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                plist.append(p)
        if not plist:
            raise ValueError("no trainable parameters")
        dev = plist[0].device
        if dev.type != "cuda":
            raise RuntimeError("FusedAdamW needs the model on the GPU")
        for p in plist:
            if p.dtype != torch.float32:
                raise TypeError("master parameters must be fp32")
        self.params = plist
        self.numel = sum(p.numel() for p in plist)
        # pad to a multiple of 64 elements per tensor so every view starts 256-B aligned
        offs, o = [], 0
        for p in plist:
            offs.append(o)
            o += (p.numel() + 63) // 64 * 64
        self.total = o
        self.offsets = offs
        self.data = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, off in zip(plist, offs):
                n = p.numel()
                self.data[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.data[off:off + n].view_as(p)
                p.grad = self.grad[off:off + n].view_as(p)

    def attach_grads(self):
        for p, off in zip(self.params, self.offsets):
            n = p.numel()
            p.grad = self.grad[off:off + n].view_as(p)

    def zero_grad(self):
        self.grad.zero_()
        self.attach_grads()


class FusedAdamW:
    """torch.optim.AdamW-compatible surface (step / zero_grad / state_dict / param_groups)."""

    def __init__(self, params, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4, max_grad_norm=None):
        self.flat = FlatParams(params)
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), tuple(betas), float(eps), float(weight_decay)
        self.max_grad_norm = max_grad_norm
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)
        self.step_count = 0
        self.last_info = None  # device tensor: [norm, clip coef, finite, -]
        self.param_groups = [dict(params=self.flat.params, lr=self.lr, betas=self.betas, eps=self.eps,
                                  weight_decay=self.weight_decay)]

    # -------------------------------------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        # grads live in the flat buffer: zero it (set_to_none would detach the views)
        self.flat.zero_grad()

    def clip_grad_norm_(self, max_norm, loss=None):
        """Computes the global grad norm and the clamped clip coefficient ON DEVICE; the
        coefficient is applied inside the next step()."""
        self.max_grad_norm = max_norm
        self.last_info = K.grad_norm(self.flat.grad, max_norm if max_norm else 0.0, loss)
        return self.last_info[0]

    def step(self, closure=None, loss=None):
        g = self.param_groups[0]
        lr = float(g["lr"])
        b1, b2 = g["betas"]
        if self.last_info is None or loss is not None:
            self.last_info = K.grad_norm(self.flat.grad, self.max_grad_norm or 0.0, loss)
        use_clip = bool(self.max_grad_norm)
        self.step_count += 1
        K.adamw(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, self.last_info, lr, b1, b2,
                g["eps"], g["weight_decay"], self.step_count, use_clip)
        self.last_info = None
        # parameters changed behind autograd's back: invalidate cached packed (bf16 / GEMM-layout) weights
        bump_param_epoch()

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "param_groups": [{k: v for k, v in self.param_groups[0].items() if k != "params"}]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.param_groups[0].update(sd["param_groups"][0])
