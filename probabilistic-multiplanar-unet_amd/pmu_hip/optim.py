"""Fused clip_grad_value_ + SGD(momentum) for the training step of PMU/train.py:65,108-110.

``FusedSGD`` has torch.optim.SGD's constructor surface (params, lr, momentum, dampening=0,
nesterov=False, weight_decay=0) plus ``clip`` (the train.py clip value, 0.1) and performs

    g = clamp(g * grad_scale, -clip, clip); buf = momentum * buf + g; p -= lr * buf

for every parameter in ONE kernel launch (pmu_sgd_clip).  buf starts at zero, which equals
torch's first-step ``buf = g.clone()``.  ``grad_scale`` (1/world_size) turns an all-reduced
gradient sum into the data-parallel mean before clipping.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from . import engine

CHUNK = 16384   # elements per block: 16 per thread, 4 float4 loads of p, g and buf in flight


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0, weight_decay=0, nesterov=False, clip=0.0):
        if dampening != 0 or weight_decay != 0 or nesterov:
            raise ValueError("FusedSGD implements the reference's SGD(lr, momentum) only (train.py:65)")
        super().__init__(params, dict(lr=lr, momentum=momentum, clip=clip))
        self._tables = {}

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict; the loaded momentum buffers replace the ones the
        kernel's cached pointer tables name."""
        super().load_state_dict(state_dict)
        self._tables.clear()

    def _table(self, plist, dev):
        key = tuple((p.data_ptr(), p.grad.data_ptr(), id(self.state[p].get("momentum_buffer"))) for p in plist)
        tab = self._tables.get(key)
        if tab is not None and all(t is self.state[p].get("momentum_buffer") for t, p in zip(tab[3], plist)):
            return tab
        ptrs, chunks = [], []
        for i, p in enumerate(plist):
            st = self.state[p]
            if "momentum_buffer" not in st or st["momentum_buffer"] is None:
                st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            assert p.is_contiguous() and p.grad.is_contiguous() and p.dtype == torch.float32
            ptrs += [p.data_ptr(), p.grad.data_ptr(), st["momentum_buffer"].data_ptr()]
            n = p.numel()
            for s in range(0, n, CHUNK):
                chunks.append((i, min(CHUNK, n - s), s))
        ptr_t = torch.tensor(ptrs, dtype=torch.int64).to(dev)
        ck = (L.PmuSgdChunk * len(chunks))(*[L.PmuSgdChunk(t, ln, st) for t, ln, st in chunks])
        ck_t = torch.frombuffer(bytearray(ck), dtype=torch.uint8).to(dev)
        tab = (ptr_t, ck_t, len(chunks), [self.state[p]["momentum_buffer"] for p in plist])
        if len(self._tables) > 8:
            self._tables.clear()
        key = tuple((p.data_ptr(), p.grad.data_ptr(), id(self.state[p]["momentum_buffer"])) for p in plist)
        self._tables[key] = tab
        return tab

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            plist = [p for p in group["params"] if p.grad is not None]
            if not plist:
                continue
            dev = plist[0].device
            ptr_t, ck_t, nck, _ = self._table(plist, dev)
            L.call("pmu_sgd_clip", ck_t.data_ptr(), nck, ptr_t.data_ptr(), float(grad_scale), float(group["lr"]),
                   float(group["momentum"]), float(group["clip"]), L.stream())
            # the kernel wrote the parameters: refresh their packed layouts in one batched launch per
            # layout, so the next forward / backward launches no pack kernel
            engine.repack(plist)
        return loss
