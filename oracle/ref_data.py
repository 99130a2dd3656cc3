"""CPU restatement of dataset_single_member.py:5-196 (WindowedAllMembersDataset_random) —
TEST INFRASTRUCTURE ONLY (parity oracle for cesm_emulator_amd.data; never imported by the product).

Only numpy / torch-CPU; the random draws use numpy's global RNG in the reference's order
(`_choose_times` draws, then `np.random.rand()` for the time reversal (:180), then
`np.random.randint` for the crop (:162-163)) so a seeded run reproduces the reference's items.
"""
from __future__ import annotations

import numpy as np
import torch


class WindowedAllMembersDatasetRef:
    def __init__(self, cond_np, tgt_np, K=5, center=True, crop_hw=None, crop_mode="random", time_reverse_p=0.5,
                 sample_mode="consecutive", window_radius=5, keep_chronology=True, causal=False,
                 allow_replace=False):
        assert cond_np.ndim == 5 and tgt_np.ndim == 5
        assert cond_np.shape == tgt_np.shape
        self.cond = cond_np.astype(np.float32)
        self.tgt = tgt_np.astype(np.float32)
        self.T, self.M, _, self.H, self.W = self.cond.shape
        if K < 2:
            raise ValueError("K must be >= 2")
        self.K, self.center = int(K), bool(center)
        if crop_hw is None:
            self.crop_h = self.crop_w = None
        else:
            self.crop_h, self.crop_w = min(int(crop_hw[0]), self.H), min(int(crop_hw[1]), self.W)
        self.crop_mode = crop_mode
        self.time_reverse_p = float(time_reverse_p)
        self.sample_mode = sample_mode
        self.window_radius = int(window_radius)
        self.keep_chronology = bool(keep_chronology)
        self.causal = bool(causal)
        self.allow_replace = bool(allow_replace)
        if self.causal and self.center:
            self.center = False
        if sample_mode == "consecutive":
            self.num_units, self.use_windows = max(1, self.T - self.K + 1), True
        else:
            self.num_units, self.use_windows = self.T, False

    def __len__(self):
        return self.num_units * self.M

    def _index_to_tm(self, idx):  # :91-102
        m, u = idx % self.M, idx // self.M
        if self.use_windows:
            t0 = u
            anchor = t0 + (self.K // 2) if self.center else t0 + self.K - 1
        else:
            anchor = u
            t0 = max(0, min(anchor - self.K // 2, self.T - self.K))
        return t0, int(np.clip(anchor, 0, self.T - 1)), m

    def _choose_times(self, t0, anchor):  # :104-150
        K = self.K
        if self.sample_mode == "consecutive":
            return np.arange(t0, t0 + K, dtype=np.int64)
        if self.sample_mode == "random_global":
            pool = np.arange(0, self.T, dtype=np.int64)
        else:
            pool = np.arange(max(0, anchor - self.window_radius), min(self.T - 1, anchor + self.window_radius) + 1,
                             dtype=np.int64)
        if self.causal:
            pool = pool[pool <= anchor]
        pool_wo = pool[pool != anchor]
        need = K - 1
        if (not self.allow_replace) and pool_wo.size < need:
            self.allow_replace = True
        if self.allow_replace:
            sampled = (np.full((need,), anchor, dtype=np.int64) if pool_wo.size == 0
                       else np.random.choice(pool_wo, size=need, replace=True))
        else:
            sampled = np.random.choice(pool_wo, size=need, replace=False)
        times = np.concatenate([sampled, np.array([anchor], dtype=np.int64)])
        if self.keep_chronology:
            times.sort()
        if self.center:
            idx_a = int(np.where(times == anchor)[0][0])
            times = np.roll(times, K // 2 - idx_a)
        else:
            times = np.array([t for t in times if t != anchor] + [anchor], dtype=np.int64)
        return times

    def _crop_coords(self, H, W):  # :152-166
        if self.crop_h is None or self.crop_w is None:
            return 0, 0, H, W
        h, w = self.crop_h, self.crop_w
        if self.crop_mode == "center":
            return max(0, (H - h) // 2), max(0, (W - w) // 2), h, w
        i = 0 if H == h else np.random.randint(0, H - h + 1)
        j = 0 if W == w else np.random.randint(0, W - w + 1)
        return i, j, h, w

    def __getitem__(self, idx):  # :168-196
        t0, anchor, m = self._index_to_tm(idx)
        times = self._choose_times(t0, anchor)
        cond_win = torch.from_numpy(self.cond[times, m]).permute(1, 0, 2, 3).contiguous()
        x0 = torch.from_numpy(self.tgt[anchor, m])
        if self.time_reverse_p > 0.0 and np.random.rand() < self.time_reverse_p:
            if self.center:
                mid = self.K // 2
                left = cond_win[:, :mid].flip(dims=(1,))
                right = cond_win[:, mid + 1:].flip(dims=(1,))
                cond_win = torch.cat([left, cond_win[:, mid:mid + 1], right], dim=1)
            else:
                cond_win = cond_win.flip(dims=(1,))
        _, K, H, W = cond_win.shape
        i, j, h, w = self._crop_coords(H, W)
        return cond_win[:, :, i:i + h, j:j + w].contiguous(), x0[:, i:i + h, j:j + w].contiguous()


def window_item(cond, tgt, item, K, h, w, center):
    """Deterministic part of __getitem__ for explicit (t0, m, anchor, reverse, i, j):
    cond/tgt are (T, M, H, W) arrays; returns (cond_win [1,K,h,w], x0 [1,h,w])."""
    t0, m, anchor, rev, i, j = item
    times = np.arange(t0, t0 + K)
    cw = np.ascontiguousarray(cond[times, m][None])  # (1,K,H,W)
    if rev:
        if center:
            mid = K // 2
            cw = np.concatenate([cw[:, :mid][:, ::-1], cw[:, mid:mid + 1], cw[:, mid + 1:][:, ::-1]], axis=1)
        else:
            cw = cw[:, ::-1]
    x0 = tgt[anchor, m][None]
    return (np.ascontiguousarray(cw[:, :, i:i + h, j:j + w]), np.ascontiguousarray(x0[:, i:i + h, j:j + w]))
