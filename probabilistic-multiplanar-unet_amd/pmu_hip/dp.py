"""Data-parallel gradient exchange overlapped with the backward (row e, configs c3/c5).

The reference trains on one device (PMU/train.py:77-117: loss / acc_steps, backward, clip, SGD);
the multi-GPU layout here is one process per GPU with a SUM all-reduce of the gradients, which
reproduces the reference's accumulated gradient exactly (train.py, tests/test_dp_gloo.py).

``BucketAllReduce`` cuts the root module's flat gradient buffer (pmu_hip.functions.
flat_grad_buffer) into contiguous buckets **in the order the backward produces the gradients**.
That order is learned, as DDP does, from the first step: the HIP backward reports every layer
whose gradient kernels it has enqueued (GradSink.flush); the first step records those reports,
all-reduces the whole buffer once after the backward, and then re-lays the buffer out in report
order (``functions.set_grad_order``).  From the second step on, bucket b holds the b-th stretch
of gradients the backward emits, so when a bucket is complete its all-reduce is issued at once
(RCCL's stream waits on an event of the compute stream at that point) and crosses xGMI while the
rest of the backward still computes (one micro-batch per rank and step, config c3's layout: with
several, autograd adds each backward's gradients into .grad only after the node's kernels have
run, so the exchange waits for the last backward and goes out whole in ``finish``).  Buckets go out strictly in index order on every rank (the
collective order must match across ranks).  Parameters the backward never reported (e.g. the
Probabilistic U-Net's ``unet.outc``, which gets no gradient) sit after the last bucket in a small
tail that ``finish`` always exchanges, so every rank issues the same collectives.  The learned
order is rank 0's, broadcast once, so a rank that ran no backward in the first step (an idle rank
of train.py's exact accumulation) agrees on it.  Gradients autograd kept outside the buffer (a
module applied twice in one graph, ``zero_grad(set_to_none=False)``) are copied into their slots
before the remaining buckets go out and copied back after.

Bucket size: xGMI is point-to-point (7 links per GPU), so a ring all-reduce is per-link bound and
gains nothing from one huge message; ~32 MB buckets keep each RCCL call well past its latency
floor while the first buckets start early in the backward.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .functions import _offsets, _slot, flat_grad_buffer, set_grad_order

DEFAULT_BUCKET_BYTES = 32 << 20


class BucketAllReduce:
    """Overlapped SUM all-reduce of ``net``'s gradients.  Usage per optimizer step::

        sync.begin()          # before the LAST backward of the step (accumulation: the others
        loss.backward()       #   just add into the .grad tensors)
        sync.finish()         # all buckets issued and waited on; grads hold the sums

    ``issued_at[b]`` is the index of the GradSink flush (counted from ``begin``) during which
    bucket b was issued, or None when ``finish`` issued it; ``flushes`` the number of flushes."""

    def __init__(self, net, bucket_bytes: int | None = None, group=None):
        if bucket_bytes is None:
            bucket_bytes = int(os.environ.get("PMU_DP_BUCKET_MB", "32")) << 20
        self.net = net
        self.group = group
        self.plist = list(net.parameters())
        self.cap = max(1, bucket_bytes // 4)
        self.buckets = None      # (lo, hi) element ranges of the buffer, backward order
        self.bucket_of = {}
        self.tail = None         # (lo, hi, members): parameters the backward never reported
        self.recording = None
        self.active = False
        self.works = []
        self.issued_at = []
        self.flushes = 0
        net.__dict__["_pmu_grad_ready"] = self._ready
        order = net.__dict__.get("_pmu_dp_order")
        if order is not None:    # a layout learned by an earlier reducer of this module
            self._build(order)

    # ---------------------------------------------------------------- layout
    def _build(self, reported):
        """Buckets over ``reported`` (parameters in backward report order); the rest form the tail."""
        ids = {id(p) for p in reported}
        rest = [p for p in self.plist if id(p) not in ids]
        set_grad_order(self.net, list(reported) + rest)
        self.net.__dict__["_pmu_dp_order"] = list(reported)
        self.buf = flat_grad_buffer(self.net, self.plist)
        offs = _offsets(self.net, self.plist)
        self.buckets, self.bucket_of = [], {}
        lo, members = 0, []
        for p in reported:
            members.append(p)
            hi = offs[id(p)] + _slot(p.numel())
            if hi - lo >= self.cap:
                self._add(lo, hi, members)
                lo, members = hi, []
        if members:
            self._add(lo, offs[id(members[-1])] + _slot(members[-1].numel()), members)
        end = self.buckets[-1][1] if self.buckets else 0
        self.tail = (end, self.buf.numel(), rest) if rest else None
        self.sizes = [0] * len(self.buckets)
        for b in self.bucket_of.values():
            self.sizes[b] += 1
        self._stale = True

    def _zero_stale(self):
        """Once after a relayout: the buffer still holds the old layout's values where the new one has
        pads and the slots of parameters without a gradient (the tail is SUM-all-reduced every step,
        so stale values there would grow by ~world per step).  A .grad that survived the relayout
        (zero_grad(set_to_none=False), a caller holding .grad across the first step) is still an
        old-layout view: it is first moved out of the buffer (a copy, exchanged like any gradient
        autograd kept outside it), so every in-buffer gradient sits at its new slot; then everything
        but those slots is zeroed."""
        self._stale = False
        buf = flat_grad_buffer(self.net, self.plist)
        offs = _offsets(self.net, self.plist)
        es = buf.element_size()
        lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * es
        inbuf = [p for p in self.plist if p.grad is not None and lo <= p.grad.data_ptr() < hi]
        moved = [p for p in inbuf if (p.grad.data_ptr() - lo) // es != offs[id(p)]]
        copies = [p.grad.detach().clone() for p in moved]   # all read before any slot is touched
        for p, c in zip(moved, copies):
            p.grad = c
        moved_ids = {id(p) for p in moved}
        keep = sorted((offs[id(p)], offs[id(p)] + p.numel()) for p in inbuf if id(p) not in moved_ids)
        pos = 0
        for a, b in keep + [(buf.numel(), buf.numel())]:
            if a > pos:
                buf[pos:a].zero_()
            pos = max(pos, b)

    def _add(self, lo, hi, members):
        b = len(self.buckets)
        self.buckets.append((lo, hi))
        for p in members:
            self.bucket_of[id(p)] = b

    # ---------------------------------------------------------------- step
    def begin(self):
        self.works = []
        self.flushes = 0
        self.active = True
        if getattr(self, "_stale", False):
            self._zero_stale()
        if self.buckets is None:
            self.recording = []
            return
        self.left = list(self.sizes)
        self.next = 0
        self.issued_at = [None] * len(self.buckets)

    def _issue_range(self, lo, hi):
        self.works.append(dist.all_reduce(self.buf[lo:hi], group=self.group, async_op=True))

    def _ready(self, params, flat=True):
        """GradSink.flush callback: ``params``' gradient kernels are enqueued.  ``flat``: into the flat
        buffer (else into tensors autograd adds to .grad later: order recorded, no bucket issued —
        those gradients are copied into their slots in ``finish``)."""
        if not self.active:
            return
        if self.recording is not None:
            seen = {id(p) for p in self.recording}
            self.recording += [p for p in params if id(p) not in seen]
            return
        if not flat:
            return
        self.flushes += 1
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is not None:
                self.left[b] -= 1
        while self.next < len(self.buckets) and self.left[self.next] <= 0:
            self.issued_at[self.next] = self.flushes - 1
            self._issue_range(*self.buckets[self.next])
            self.next += 1

    @property
    def issued_in_backward(self) -> int:
        return sum(1 for i in self.issued_at if i is not None)

    def _agree(self, reported):
        """Rank 0's report order, broadcast (every rank must cut the same buckets; an idle rank
        recorded nothing)."""
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return reported
        dev = self.buf.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        pos = {id(p): i for i, p in enumerate(self.plist)}
        t = torch.full((len(self.plist),), -1, dtype=torch.int64)
        t[:len(reported)] = torch.tensor([pos[id(p)] for p in reported], dtype=torch.int64)
        t = t.to(dev)
        dist.broadcast(t, 0, group=self.group)
        return [self.plist[i] for i in t.cpu().tolist() if i >= 0]

    def finish(self, idle: bool = False):
        """Issue what is left, wait, and leave the sums in the gradients.  ``idle``: this rank ran
        no backward this step (fewer micro-batches than ranks); it contributes zeros and adopts
        the summed gradients of every parameter the backward reports."""
        if not self.active:
            raise RuntimeError("BucketAllReduce.finish() without begin()")
        self.active = False
        self.buf = buf = flat_grad_buffer(self.net, self.plist)
        offs = _offsets(self.net, self.plist)
        lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * buf.element_size()
        foreign = [p for p in self.plist if p.grad is not None and not lo <= p.grad.data_ptr() < hi]
        if idle:
            if any(p.grad is not None for p in self.plist):
                raise RuntimeError("BucketAllReduce.finish(idle=True) with gradients present")
            buf.zero_()
        slot = lambda p: buf[offs[id(p)]:offs[id(p)] + p.numel()].view_as(p)  # noqa: E731
        if self.recording is not None:
            # first step: the whole buffer in one all-reduce, then the learned layout
            for p in foreign:
                slot(p).copy_(p.grad)
            self._issue_range(0, buf.numel())
            reported = self._agree(self.recording)
            self.recording = None
            self._wait(foreign, slot, reported if idle else ())
            if reported:
                self._build(reported)
            return
        if foreign:
            issued = {id(p) for b in range(self.next) for p in self.plist if self.bucket_of.get(id(p)) == b}
            if any(id(p) in issued for p in foreign):
                # a bucket already in flight would race with autograd copying it into a fresh .grad
                raise RuntimeError("gradients were not adopted from the flat buffer while buckets were in flight")
            for p in foreign:
                slot(p).copy_(p.grad)
        while self.next < len(self.buckets):
            self._issue_range(*self.buckets[self.next])
            self.next += 1
        if self.tail is not None:   # always, so every rank issues the same collectives
            self._issue_range(self.tail[0], self.tail[1])
        self._wait(foreign, slot, self.net.__dict__["_pmu_dp_order"] if idle else ())

    def _wait(self, foreign, slot, adopt):
        for w in self.works:
            w.wait()
        self.works = []
        for p in foreign:   # grads autograd kept outside the buffer get their sums back
            p.grad.copy_(slot(p))
        for p in adopt:     # idle rank: the summed gradients of the busy ranks
            p.grad = slot(p)

    def detach(self):
        self.net.__dict__.pop("_pmu_grad_ready", None)
