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
        params = list(params)
        # every parameter passed in, frozen ones included: torch.optim indexes its state_dict by this order
        self.all_params = params
        self._index = {}
        for i, p in enumerate(params):
            self._index.setdefault(id(p), i)
        self.flat = FlatParams(params)
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), tuple(betas), float(eps), float(weight_decay)
        self.max_grad_norm = max_grad_norm
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)
        # step counter on the device: the AdamW launch advances it only for a finite step, so a skipped
        # (non-finite) step leaves bias corrections and the saved "step" consistent with exp_avg/exp_avg_sq
        self._step_dev = torch.zeros(1, dtype=torch.int32, device=self.flat.data.device)
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
        K.adamw(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, self.last_info, lr, b1, b2,
                g["eps"], g["weight_decay"], self._step_dev, use_clip)
        self.last_info = None
        # parameters changed behind autograd's back: invalidate cached packed (bf16 / GEMM-layout) weights
        bump_param_epoch()

    @property
    def step_count(self):
        """number of applied (finite) steps; reading it synchronises with the device"""
        return int(self._step_dev.item())

    @step_count.setter
    def step_count(self, n):
        self._step_dev.fill_(int(n))

    def state_dict(self):
        """torch.optim.AdamW layout — what train.py:1164 stores under "optimizer" — so checkpoints
        round-trip with the reference: state[i] for the i-th parameter passed in (frozen ones, e.g. the
        rotary freqs, carry no state), group keys as the installed torch's AdamW writes them."""
        state = {}
        nstep = self.step_count
        if nstep > 0:
            for p, off in zip(self.flat.params, self.flat.offsets):
                n = p.numel()
                state[self._index[id(p)]] = {
                    "step": torch.tensor(float(nstep)),
                    "exp_avg": self.exp_avg[off:off + n].view_as(p).clone(),
                    "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p).clone()}
        group = dict(_adamw_group_defaults())
        group.update({k: v for k, v in self.param_groups[0].items() if k != "params"})
        group["betas"] = tuple(group["betas"])
        group["params"] = list(range(len(self.all_params)))
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        """Accepts torch.optim.AdamW state dicts (reference checkpoints) and the flat form of earlier
        versions of this class."""
        if "state" not in sd:  # flat form
            self.step_count = int(sd["step"])
            self.exp_avg.copy_(sd["exp_avg"])
            self.exp_avg_sq.copy_(sd["exp_avg_sq"])
            self.param_groups[0].update(sd["param_groups"][0])
            return
        g = sd["param_groups"][0]
        if len(g["params"]) != len(self.all_params):
            raise ValueError(f"optimizer state has {len(g['params'])} parameters, model has {len(self.all_params)}")
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in g:
                self.param_groups[0][k] = tuple(g[k]) if k == "betas" else g[k]
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        steps = set()
        with torch.no_grad():
            for p, off in zip(self.flat.params, self.flat.offsets):
                st = sd["state"].get(self._index[id(p)], sd["state"].get(str(self._index[id(p)])))
                if not st:
                    continue
                n = p.numel()
                self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"per-parameter step counts differ ({sorted(steps)}); the fused step needs one")
        self.step_count = steps.pop() if steps else 0


_GROUP_DEFAULTS = None


def _adamw_group_defaults():
    """param_group keys/defaults of the installed torch.optim.AdamW (the de-facto pinned version)."""
    global _GROUP_DEFAULTS
    if _GROUP_DEFAULTS is None:
        g = torch.optim.AdamW([torch.zeros(1, requires_grad=True)]).param_groups[0]
        _GROUP_DEFAULTS = {k: v for k, v in g.items() if k != "params"}
    return _GROUP_DEFAULTS
