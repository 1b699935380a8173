"""Data-parallel gradient exchange overlapped with the backward (row e, configs c3/c5).

The reference trains on one device (PMU/train.py:77-117: loss / acc_steps, backward, clip, SGD);
the multi-GPU layout here is one process per GPU with a SUM all-reduce of the gradients, which
reproduces the reference's accumulated gradient exactly (train.py, tests/test_dp_gloo.py).

``BucketAllReduce`` splits the root module's flat gradient buffer (pmu_hip.functions.
flat_grad_buffer: parameters in registration order) into contiguous buckets taken from its END,
i.e. in the order the backward produces them (head, decoder from the top level down, deepest
encoder level, ..., first encoder block).  The HIP backward reports every layer whose gradient
kernels it has enqueued (GradSink.flush); when a bucket is complete its all-reduce is issued at
once (RCCL's stream waits on an event of the compute stream at that point), so the exchange of
the decoder's and the deep levels' gradients runs while the shallow levels' backward still
computes.  Buckets are issued strictly in index order on every rank (the collective order must
match across ranks); ``finish`` issues whatever is left (parameters that got no gradient keep
stale slots, which the optimizer ignores since their .grad is None) and waits.

Bucket size: xGMI is point-to-point (7 links per GPU), so a ring all-reduce is per-link bound and
gains nothing from one huge message; ~32 MB buckets keep each RCCL call well past its latency
floor while the first buckets start early in the backward.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .functions import _offsets, flat_grad_buffer

DEFAULT_BUCKET_BYTES = 32 << 20


class BucketAllReduce:
    """Overlapped SUM all-reduce of ``net``'s gradients.  Usage per optimizer step::

        sync.begin()          # before the LAST backward of the step (accumulation: the others
        loss.backward()       #   just add into the flat buffer)
        sync.finish()         # all buckets issued and waited on; grads hold the sums
    """

    def __init__(self, net, bucket_bytes: int | None = None, group=None):
        if bucket_bytes is None:
            bucket_bytes = int(os.environ.get("PMU_DP_BUCKET_MB", "32")) << 20
        self.net = net
        self.group = group
        self.plist = list(net.parameters())
        self.buf = flat_grad_buffer(net, self.plist)
        offs = _offsets(net, self.plist)
        cap = max(1, bucket_bytes // self.buf.element_size())
        self.buckets = []      # (lo, hi) element ranges of buf, backward order
        self.bucket_of = {}
        members = []
        hi = self.buf.numel()
        for p in reversed(self.plist):
            members.append(p)
            lo = offs[id(p)]
            if hi - lo >= cap:
                self._add(lo, hi, members)
                members, hi = [], lo
        if members:
            self._add(0, hi, members)
        self.sizes = [0] * len(self.buckets)
        for b in self.bucket_of.values():
            self.sizes[b] += 1
        self.active = False
        self.left = []
        self.next = 0
        self.works = []
        self.issued_in_backward = 0
        net.__dict__["_pmu_grad_ready"] = self._ready

    def _add(self, lo, hi, members):
        b = len(self.buckets)
        self.buckets.append((lo, hi))
        for p in members:
            self.bucket_of[id(p)] = b

    def begin(self):
        self.left = list(self.sizes)
        self.next = 0
        self.works = []
        self.issued_in_backward = 0
        self.active = True

    def _issue(self, b):
        lo, hi = self.buckets[b]
        self.works.append(dist.all_reduce(self.buf[lo:hi], group=self.group, async_op=True))

    def _ready(self, params):
        """GradSink.flush callback: ``params``' gradient kernels are enqueued."""
        if not self.active:
            return
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is not None:
                self.left[b] -= 1
        while self.next < len(self.buckets) and self.left[self.next] <= 0:
            self._issue(self.next)
            self.next += 1
            self.issued_in_backward += 1

    def finish(self):
        if not self.active:
            raise RuntimeError("BucketAllReduce.finish() without begin()")
        self.active = False
        lo, hi = self.buf.data_ptr(), self.buf.data_ptr() + self.buf.numel() * self.buf.element_size()
        foreign = [p for p in self.plist if p.grad is not None and not lo <= p.grad.data_ptr() < hi]
        if foreign and self.next > 0:
            # a bucket already in flight would race with autograd copying it into a fresh .grad
            raise RuntimeError("gradients were not adopted from the flat buffer while buckets were in flight")
        while self.next < len(self.buckets):
            self._issue(self.next)
            self.next += 1
        if foreign:
            # grads that autograd accumulated outside the buffer (zero_grad(set_to_none=False)):
            # one flattened bucket, issued after the buffer's buckets on every rank
            flat = torch.cat([p.grad.reshape(-1) for p in foreign])
            self.works.append(dist.all_reduce(flat, group=self.group, async_op=True))
        for w in self.works:
            w.wait()
        self.works = []
        if foreign:
            off = 0
            for p in foreign:
                n = p.grad.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n

    def detach(self):
        self.net.__dict__.pop("_pmu_grad_ready", None)
