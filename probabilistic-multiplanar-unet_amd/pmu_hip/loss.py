"""The training losses on HIP kernels (row a6): drop-ins for the torch criteria the reference builds.

  BCELoss           nn.BCELoss on the sigmoid head (UNetTrainer, PMU/trainer/unet_trainer.py:23,33-37)
  CrossEntropyLoss  nn.CrossEntropyLoss on the logits (UNetTrainer n_classes > 1; ProbabilisticUnet.elbo
                    with reduction 'none' summed, probabilistic_unet.py:286-304)

Same constructors and reductions as torch's; the forward is one deterministic streaming reduction
(pmu_bce_fwd / pmu_ce_fwd), the backward one elementwise kernel scaled on the device by the upstream
gradient (pmu_bce_bwd / pmu_ce_bwd): no host synchronisation.  Per-class weights, label smoothing
and probabilistic (float) CE targets are not used by the reference and are rejected.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as L

_RED = {"none": 0, "mean": 1, "sum": 2}


def _red(reduction):
    if reduction not in _RED:
        raise ValueError(f"reduction {reduction!r}")
    return _RED[reduction]


def _dev_check(name, *ts):
    for t in ts:
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise RuntimeError(f"{name} runs on the MI355X HIP path only (there is no CPU fallback)")


class _BCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, t, red):
        yc, tc = y.detach().contiguous().float(), t.detach().contiguous().float()
        n = yc.numel()
        s = L.stream()
        if red == 0:
            loss = torch.empty_like(yc)
            L.call("pmu_bce_fwd", yc.data_ptr(), tc.data_ptr(), n, 0, loss.data_ptr(), None, None, s)
        else:
            loss = torch.empty((), dtype=torch.float32, device=y.device)
            ws = torch.empty(L.lib().pmu_loss_ws(n) // 8, dtype=torch.float64, device=y.device)
            L.call("pmu_bce_fwd", yc.data_ptr(), tc.data_ptr(), n, red, loss.data_ptr(), ws.data_ptr(), None, s)
        ctx.save_for_backward(yc, tc)
        ctx.red = red
        return loss

    @staticmethod
    def backward(ctx, g):
        yc, tc = ctx.saved_tensors
        gc = g.detach().contiguous().float()
        dy = torch.empty_like(yc)
        L.call("pmu_bce_bwd", yc.data_ptr(), tc.data_ptr(), yc.numel(), ctx.red, gc.data_ptr(), dy.data_ptr(),
               L.stream())
        return dy, None, None


class _CE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, red, ignore):
        xc = x.detach().contiguous().float()
        tc = t.detach().contiguous().long()
        N, K = xc.shape[0], xc.shape[1]
        HW = xc[0, 0].numel()
        if tc.numel() != N * HW:
            raise RuntimeError(f"CrossEntropyLoss: target {tuple(t.shape)} does not match input {tuple(x.shape)}")
        s = L.stream()
        count = torch.empty((), dtype=torch.float32, device=x.device)
        if red == 0:
            loss = torch.empty(tc.shape, dtype=torch.float32, device=x.device)
            L.call("pmu_ce_fwd", xc.data_ptr(), tc.data_ptr(), N, K, HW, 0, ignore, loss.data_ptr(), None, None, s)
        else:
            loss = torch.empty((), dtype=torch.float32, device=x.device)
            ws = torch.empty(L.lib().pmu_loss_ws(N * HW) // 8, dtype=torch.float64, device=x.device)
            L.call("pmu_ce_fwd", xc.data_ptr(), tc.data_ptr(), N, K, HW, red, ignore, loss.data_ptr(), ws.data_ptr(),
                   count.data_ptr(), s)
        ctx.save_for_backward(xc, tc, count)
        ctx.red, ctx.ignore = red, ignore
        return loss

    @staticmethod
    def backward(ctx, g):
        xc, tc, count = ctx.saved_tensors
        gc = g.detach().contiguous().float()
        dx = torch.empty_like(xc)
        N, K = xc.shape[0], xc.shape[1]
        L.call("pmu_ce_bwd", xc.data_ptr(), tc.data_ptr(), N, K, xc[0, 0].numel(), ctx.red, ctx.ignore, gc.data_ptr(),
               count.data_ptr(), dx.data_ptr(), L.stream())
        return dx, None, None, None


class BCELoss(nn.BCELoss):
    """nn.BCELoss(weight=None, reduction='mean') on HIP kernels."""

    def forward(self, input, target):
        if self.weight is not None:
            raise NotImplementedError("BCELoss(weight=...) is not used by the reference")
        if input.shape != target.shape:
            raise ValueError(f"Using a target size ({target.shape}) that is different to the input size ({input.shape})")
        _dev_check("BCELoss", input, target)
        return _BCE.apply(input, target, _red(self.reduction))


class CrossEntropyLoss(nn.CrossEntropyLoss):
    """nn.CrossEntropyLoss(weight=None, ignore_index=-100, reduction='mean', label_smoothing=0) on HIP
    kernels; class-index targets (N, *) for logits (N, C, *)."""

    def forward(self, input, target):
        if self.weight is not None or self.label_smoothing != 0.0:
            raise NotImplementedError("CrossEntropyLoss weight / label_smoothing are not used by the reference")
        if target.is_floating_point():
            raise NotImplementedError("CrossEntropyLoss with class-probability targets is not used by the reference")
        _dev_check("CrossEntropyLoss", input, target)
        return _CE.apply(input, target, _red(self.reduction), int(self.ignore_index))
