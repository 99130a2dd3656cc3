"""Training data path: dataset_single_member.py's windowed sampler + the train.py load → device copy.

Two device feeds, both producing the reference's batches `cond [B,1,K,h,w]`, `x0 [B,1,h,w]`:

* `DeviceWindowLoader` — the z-scored (T, M, H, W) fields live in HBM (2.2 GB each for the full
  CESM2-LE grid, a rounding error in 288 GB); per batch the host only draws the item parameters
  (t0, member, anchor, reverse flag, crop offsets — same numpy RNG order as the reference
  `__getitem__`) and the `cesm_window_gather` kernel assembles the batch on device.
* `PinnedWindowLoader` — host-resident fields: items are gathered on the host into pinned
  double-buffers and copied with non-blocking H2D copies on a side stream, overlapped with the
  previous step's compute and ordered with events.

`load_cond_and_target` restates train.py:600-650 for .npy/.npz inputs (NetCDF readers — xarray,
netCDF4 — are not in this image); z-scoring uses the reference's single global mean/std.
"""
from __future__ import annotations

import numpy as np
import torch

from . import kernels as K


def zscore(a):
    """train.py:640-646: one global mean/std per array (std + 1e-8)."""
    m, s = float(a.mean()), float(a.std() + 1e-8)
    return ((a - m) / s).astype(np.float32), m, s


def load_cond_and_target(cond_file, target_file, cond_var=None, target_var=None, normalize=True):
    """(T, M, H, W) float32 arrays from .npy / .npz files (key = var name, or the only array)."""
    def _load(path, var):
        if str(path).endswith(".nc"):
            raise RuntimeError("NetCDF input needs xarray/netCDF4, which this image lacks: convert to .npz")
        obj = np.load(path, allow_pickle=False)
        if isinstance(obj, np.lib.npyio.NpzFile):
            arr = obj[var] if var is not None else obj[obj.files[0]]
        else:
            arr = obj
        arr = np.asarray(arr, dtype=np.float32)
        if arr.ndim == 5:
            arr = arr[:, :, 0]
        if arr.ndim != 4:
            raise ValueError(f"expected (T, M, H, W) data in {path}, got shape {arr.shape}")
        return arr

    c = _load(cond_file, cond_var)
    t = _load(target_file, target_var)
    if normalize:
        c, _, _ = zscore(c)
        t, _, _ = zscore(t)
    return c, t


class WindowSampler:
    """Item-parameter draws of WindowedAllMembersDataset_random (consecutive sample mode):
    dataset_single_member.py:91-102 (index -> t0/anchor/member), :180 (time reversal draw),
    :156-166 (crop draw).  Uses numpy's global RNG in the reference's per-item order."""

    def __init__(self, T, M, H, W, K, center=True, crop_hw=None, crop_mode="random", time_reverse_p=0.5,
                 sample_mode="consecutive"):
        if sample_mode != "consecutive":
            raise NotImplementedError("the device window gather implements sample_mode='consecutive' "
                                      "(the mode both reference configs use)")
        if K < 2:
            raise ValueError("K must be >= 2")
        self.T, self.M, self.H, self.W, self.K = T, M, H, W, int(K)
        self.center = bool(center)
        self.crop = None if not crop_hw else (min(int(crop_hw[0]), H), min(int(crop_hw[1]), W))
        self.crop_mode = crop_mode
        self.p = float(time_reverse_p)
        self.num_units = max(1, T - self.K + 1)

    def __len__(self):
        return self.num_units * self.M

    @property
    def hw(self):
        return self.crop if self.crop else (self.H, self.W)

    def item(self, idx):
        m, t0 = idx % self.M, idx // self.M
        anchor = t0 + (self.K // 2) if self.center else t0 + self.K - 1
        anchor = int(np.clip(anchor, 0, self.T - 1))
        rev = 1 if (self.p > 0.0 and np.random.rand() < self.p) else 0
        i = j = 0
        if self.crop:
            h, w = self.crop
            if self.crop_mode == "center":
                i, j = max(0, (self.H - h) // 2), max(0, (self.W - w) // 2)
            else:
                i = 0 if self.H == h else np.random.randint(0, self.H - h + 1)
                j = 0 if self.W == w else np.random.randint(0, self.W - w + 1)
        return [t0, m, anchor, rev, i, j]

    def items(self, indices):
        return np.asarray([self.item(int(k)) for k in indices], dtype=np.int64).reshape(-1, 6)


def host_gather(cond, tgt, items, K, h, w, center, out_c, out_x):
    """Host-side batch assembly for the pinned path: out_c [n,1,K,h,w], out_x [n,1,h,w] (numpy
    views of pinned buffers) from (T,M,H,W) fields and item rows (t0, m, anchor, rev, i, j)."""
    for n, (t0, m, anchor, rev, i, j) in enumerate(items):
        cw = cond[t0:t0 + K, m, i:i + h, j:j + w]
        if rev:
            if center:
                mid = K // 2
                cw = np.concatenate([cw[:mid][::-1], cw[mid:mid + 1], cw[mid + 1:][::-1]], axis=0)
            else:
                cw = cw[::-1]
        out_c[n, 0] = cw
        out_x[n, 0] = tgt[anchor, m, i:i + h, j:j + w]


def shard_indices(n, batch_size, rank=0, world=1, shuffle=True, seed=0, epoch=0, drop_last=False):
    """DistributedSampler semantics (train.py:1002): seeded permutation per epoch, padded to a
    multiple of world, rank-strided; then cut into batches."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    total = -(-n // world) * world
    idx = (idx + idx[: total - n])[:total] if total > n else idx
    mine = idx[rank:total:world]
    batches = [mine[k:k + batch_size] for k in range(0, len(mine), batch_size)]
    if drop_last and batches and len(batches[-1]) < batch_size:
        batches = batches[:-1]
    return batches


class DeviceWindowLoader:
    """HBM-resident fields + device gather kernel; iterate -> (cond [B,1,K,h,w], x0 [B,1,h,w])."""

    def __init__(self, cond, tgt, K, batch_size, device, center=True, crop_hw=None, crop_mode="random",
                 time_reverse_p=0.5, shuffle=True, seed=0, rank=0, world=1):
        cond = np.asarray(cond, dtype=np.float32)
        tgt = np.asarray(tgt, dtype=np.float32)
        if cond.ndim == 5:
            cond, tgt = cond[:, :, 0], tgt[:, :, 0]
        T, M, H, W = cond.shape
        self.sampler = WindowSampler(T, M, H, W, K, center, crop_hw, crop_mode, time_reverse_p)
        self.cond = torch.from_numpy(np.ascontiguousarray(cond)).to(device)
        self.tgt = torch.from_numpy(np.ascontiguousarray(tgt)).to(device)
        self.bs, self.device = batch_size, device
        self.shuffle, self.seed, self.rank, self.world = shuffle, seed, rank, world
        self.epoch = 0
        self._items_host = torch.empty((batch_size, 6), dtype=torch.int64).pin_memory()

    def set_epoch(self, e):
        self.epoch = e

    def __len__(self):
        return len(shard_indices(len(self.sampler), self.bs, self.rank, self.world, False))

    def batch(self, indices):
        it = self.sampler.items(indices)
        n = it.shape[0]
        host = self._items_host[:n]
        host.copy_(torch.from_numpy(it))
        dev_items = host.to(self.device, non_blocking=True)
        h, w = self.sampler.hw
        return K.window_gather(self.cond, self.tgt, dev_items, self.sampler.K, h, w, self.sampler.center)

    def __iter__(self):
        for b in shard_indices(len(self.sampler), self.bs, self.rank, self.world, self.shuffle, self.seed,
                               self.epoch):
            cw, x0 = self.batch(b)
            yield cw, x0


class PinnedWindowLoader:
    """Host-resident fields; host gather into pinned double-buffers, H2D on a side stream."""

    def __init__(self, cond, tgt, K, batch_size, device, center=True, crop_hw=None, crop_mode="random",
                 time_reverse_p=0.5, shuffle=True, seed=0, rank=0, world=1):
        cond = np.asarray(cond, dtype=np.float32)
        tgt = np.asarray(tgt, dtype=np.float32)
        if cond.ndim == 5:
            cond, tgt = cond[:, :, 0], tgt[:, :, 0]
        self.cond, self.tgt = cond, tgt
        T, M, H, W = cond.shape
        self.sampler = WindowSampler(T, M, H, W, K, center, crop_hw, crop_mode, time_reverse_p)
        self.bs, self.device = batch_size, device
        self.shuffle, self.seed, self.rank, self.world = shuffle, seed, rank, world
        self.epoch = 0
        h, w = self.sampler.hw
        self.stream = torch.cuda.Stream(device=device)
        self.host = [(torch.empty((batch_size, 1, K, h, w)).pin_memory(),
                      torch.empty((batch_size, 1, h, w)).pin_memory()) for _ in range(2)]
        self.dev = [(torch.empty((batch_size, 1, K, h, w), device=device),
                     torch.empty((batch_size, 1, h, w), device=device)) for _ in range(2)]
        self.done = [None, None]

    def set_epoch(self, e):
        self.epoch = e

    def _fill_host(self, slot, items):
        hc, hx = self.host[slot]
        h, w = self.sampler.hw
        host_gather(self.cond, self.tgt, items, self.sampler.K, h, w, self.sampler.center, hc.numpy(), hx.numpy())

    def __iter__(self):
        batches = shard_indices(len(self.sampler), self.bs, self.rank, self.world, self.shuffle, self.seed,
                                self.epoch)
        main = torch.cuda.current_stream(self.device)

        def issue(k):
            slot = k % 2
            items = self.sampler.items(batches[k])
            if self.done[slot] is not None:
                self.done[slot].synchronize()  # host buffer free once its previous copy finished
            self._fill_host(slot, items)
            n = items.shape[0]
            with torch.cuda.stream(self.stream):
                self.stream.wait_stream(main)  # device buffer no longer read by compute
                dc, dx = self.dev[slot]
                hc, hx = self.host[slot]
                dc[:n].copy_(hc[:n], non_blocking=True)
                dx[:n].copy_(hx[:n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.done[slot] = ev
            return slot, n

        if not batches:
            return
        pending = issue(0)
        for k in range(len(batches)):
            slot, n = pending
            main.wait_event(self.done[slot])
            if k + 1 < len(batches):
                pending = issue(k + 1)  # overlaps the consumer's compute on batch k
            dc, dx = self.dev[slot]
            yield dc[:n], dx[:n]
