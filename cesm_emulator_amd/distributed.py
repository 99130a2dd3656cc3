"""Data parallelism: one process per GPU, RCCL (torch.distributed "nccl" backend) over xGMI.

Replaces the reference's DDP wrapper (train.py:1075-1076) and setup (train.py:207-221).  The
reference never arms DDP's reducer (it calls the unwrapped module), so its ranks
train independent replicas; here gradients ARE averaged, making an N-rank step equal to a 1-rank
step on the concatenated batch (per-sample GroupNorm/LayerNorm => no cross-sample statistics).

Gradients live in ONE flat fp32 buffer (FusedAdamW / FlatParams), so the exchange is a few large
bucketed all-reduces issued on a dedicated communication stream, sized for xGMI's point-to-point
rings (32 MB buckets: 35 M params = 140 MB -> 5 buckets).  The average is folded into the
all-reduce via pre-scaling the bucket by 1/world on the communication stream.

Overlap with the backward: `arm()` hands the network a readiness hook.
The HIP backward walks the modules in reverse construction order, which is also reverse flat-buffer
order, and calls the hook after each level.  Once every parameter at or above a bucket's start
offset is final, that bucket's all-reduce is enqueued on the communication stream behind an event
on the compute stream, so RCCL moves the deep levels' gradients while the shallow levels' backward
still runs.  The shared accumulators (time MLP, rel-pos table) sit at the front of the buffer and
go last, in `finish()`.
"""
from __future__ import annotations

import os
from datetime import timedelta

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def setup(backend=None, timeout_min=30):
    """train.py:207-221 equivalent: env:// rendezvous when WORLD_SIZE > 1."""
    rank, local, world = env_rank()
    if world == 1 or not dist.is_available():
        return rank, local, world
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, init_method="env://", timeout=timedelta(minutes=timeout_min))
    return rank, local, world


def is_dist():
    return dist.is_available() and dist.is_initialized()


class GradAllReducer:
    """Bucketed average of a flat gradient buffer across ranks."""

    def __init__(self, bucket_bytes=32 << 20, use_side_stream=True):
        self.world = dist.get_world_size() if is_dist() else 1
        self.rank = dist.get_rank() if is_dist() else 0
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.side = use_side_stream
        self._stream = None
        self._armed = None
        # timing = True: every overlapped bucket is bracketed by HIP events on the communication stream (the pre-scale
        # and the all-reduce, which the stream waits for), so bench.py can report the measured all-reduce time per step
        self.timing = False
        self._events = []  # (start, end, bytes)

    def buckets(self, n):
        return [(s, min(n, s + self.bucket_elems)) for s in range(0, n, self.bucket_elems)]

    def allreduce_grads(self, flat_grad):
        if self.world == 1:
            return
        flat_grad.mul_(1.0 / self.world)
        if flat_grad.is_cuda and self.side:
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=flat_grad.device)
            main = torch.cuda.current_stream(flat_grad.device)
            self._stream.wait_stream(main)
            with torch.cuda.stream(self._stream):
                works = [dist.all_reduce(flat_grad[a:b], op=dist.ReduceOp.SUM, async_op=True)
                         for a, b in self.buckets(flat_grad.numel())]
                for w in works:
                    w.wait()
            main.wait_stream(self._stream)
        else:
            for a, b in self.buckets(flat_grad.numel()):
                dist.all_reduce(flat_grad[a:b], op=dist.ReduceOp.SUM)

    def pop_timing(self):
        """(total all-reduce ms, bucket count, bytes) of the buckets timed since the last call (synchronizes)"""
        if not self._events:
            return 0.0, 0, 0
        self._events[-1][1].synchronize()
        ms = sum(a.elapsed_time(b) for a, b, _ in self._events)
        n, nbytes = len(self._events), sum(x for _, _, x in self._events)
        self._events = []
        return ms, n, nbytes

    def broadcast_params(self, flat_params, src=0):
        """Initial replica sync (what DDP's constructor does at train.py:1076)."""
        if self.world > 1:
            dist.broadcast(flat_params, src=src)

    # ------------------------------------------------------------------ overlapped path
    def _comm(self, device):
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=device)
        return self._stream

    def arm(self, net, flat):
        """Reduce buckets during the coming backward.  `net` is the module whose backward calls
        `net._grad_ready(params, extra_stream)`; `flat` has .params / .offsets / .grad (FlatParams).
        Buckets are cut from the END of the buffer, the order the backward finalises it."""
        if self.world == 1:
            return
        g = flat.grad
        ends = {}
        for p, off in zip(flat.params, flat.offsets):
            ends[id(p)] = off + p.numel()
        self._armed = dict(grad=g, total=g.numel(), ends=ends, pending=set(ends), lo=g.numel(), works=[])
        net._grad_ready = self.ready

    def _issue(self, a, b, streams):
        st = self._armed
        chunk = st["grad"][a:b]
        if chunk.is_cuda and self.side:
            comm = self._comm(chunk.device)
            comm.wait_stream(torch.cuda.current_stream(chunk.device))
            for s in streams:
                if s is not None:
                    comm.wait_stream(s)
            with torch.cuda.stream(comm):
                ev = None
                if self.timing:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record(comm)
                chunk.mul_(1.0 / self.world)
                w = dist.all_reduce(chunk, op=dist.ReduceOp.SUM, async_op=True)
                if ev is not None:
                    w.wait()  # the communication stream waits for the collective: the end event follows it
                    ev[1].record(comm)
                    self._events.append((ev[0], ev[1], chunk.numel() * chunk.element_size()))
                st["works"].append(w)
        else:
            chunk.mul_(1.0 / self.world)
            dist.all_reduce(chunk, op=dist.ReduceOp.SUM)

    def ready(self, params, extra_stream=None):
        """Hook: `params` have final gradients (enqueued on the current stream / extra_stream)."""
        st = self._armed
        if st is None:
            return
        for p in params:
            st["pending"].discard(id(p))
        ready_from = max((st["ends"][i] for i in st["pending"]), default=0)
        streams = (extra_stream,)
        while st["lo"] > 0:
            b = st["lo"]
            a = max(0, b - self.bucket_elems)
            if a < ready_from:
                break
            self._issue(a, b, streams)
            st["lo"] = a

    def finish(self, net=None, extra_stream=None):
        """Reduce whatever is left, then order the compute stream after every bucket."""
        st = self._armed
        if st is None:
            return
        st["pending"].clear()
        self.ready((), extra_stream)
        for w in st["works"]:
            w.wait()
        g = st["grad"]
        if g.is_cuda and self.side and self._stream is not None:
            torch.cuda.current_stream(g.device).wait_stream(self._stream)
        self._armed = None
        if net is not None and getattr(net, "_grad_ready", None) is not None:
            net._grad_ready = None


class XgmiModelReducer(GradAllReducer):
    """One-GPU measurement of the overlapped data-parallel step (a measurement aid, not a training path): the same
    bucketing, readiness hook and communication stream as GradAllReducer, but each bucket's RCCL all-reduce is
    replaced by `cesm_hold_cus` -- `cus` blocks that each occupy a whole CU on the communication stream for the
    bucket's modelled ring all-reduce time on `world` GPUs, 2 (world - 1) / world * bytes / busbw_gbs (xGMI: RCCL's
    bus bandwidth for large all-reduces on one 8-GPU node).  The gradients are left as they are (scaled by 1.0, the
    same pre-scale kernel), so the step trains exactly like the 1-GPU step and only the timing differs.
    tools/overlap_sim.py compares it with the plain step."""

    def __init__(self, world=8, cus=32, busbw_gbs=300.0, bucket_bytes=32 << 20):
        super().__init__(bucket_bytes=bucket_bytes, use_side_stream=True)
        self.model_world, self.cus, self.busbw = int(world), int(cus), float(busbw_gbs)
        self.world = 1 if self.model_world <= 1 else self.model_world  # arms the hook (GradAllReducer.arm)
        self.issued_us = []

    def bucket_us(self, nbytes):
        w = self.model_world
        return 2.0 * (w - 1) / w * nbytes / (self.busbw * 1e3)

    def _issue(self, a, b, streams):
        from ._lib import call
        st = self._armed
        chunk = st["grad"][a:b]
        comm = self._comm(chunk.device)
        comm.wait_stream(torch.cuda.current_stream(chunk.device))
        for s in streams:
            if s is not None:
                comm.wait_stream(s)
        us = self.bucket_us(chunk.numel() * chunk.element_size())
        self.issued_us.append(us)
        with torch.cuda.stream(comm):
            chunk.mul_(1.0)
            call("cesm_hold_cus", self.cus, float(us), comm.cuda_stream)

    def allreduce_grads(self, flat_grad):
        """the non-overlapped form: every bucket held on the compute stream after the backward"""
        from ._lib import call
        for a, b in self.buckets(flat_grad.numel()):
            us = self.bucket_us((b - a) * flat_grad.element_size())
            self.issued_us.append(us)
            flat_grad[a:b].mul_(1.0)
            call("cesm_hold_cus", self.cus, float(us), torch.cuda.current_stream(flat_grad.device).cuda_stream)

    def broadcast_params(self, flat_params, src=0):
        return
