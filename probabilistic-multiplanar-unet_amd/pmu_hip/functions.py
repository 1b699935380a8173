"""Autograd bridge: one torch.autograd.Function per fused network, backed by pmu_hip.engine.

The reference builds one autograd node per PyTorch op (~90 for the 5-level U-Net); here the
whole U-Net forward is a single node whose backward replays the stack in reverse on the HIP
kernels and returns every parameter gradient at once.
"""
from __future__ import annotations

import torch

from . import engine


class UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net, x, *params):
        out, st = engine.unet_forward(net, x, net.training)
        ctx.net = net
        ctx.st = st
        ctx.nparams = len(params)
        return out

    @staticmethod
    def backward(ctx, dy):
        net = ctx.net
        plist = list(net.parameters())
        # When every .grad is None (zero_grad(set_to_none=True)), the kernels write straight into
        # fresh views of one persistent flat buffer; autograd then adopts those views as .grad,
        # so gradients are contiguous for one all-reduce and pointer-stable for the fused SGD.
        use_flat = all(p.grad is None for p in plist)
        if use_flat:
            attach_flat_grad_views(net, plist)
        grads = engine.unet_backward(net, ctx.st, dy, sink_views=use_flat)
        net._pmu_grad_views = None
        ctx.st = None
        return (None, None) + tuple(grads.get(p) for p in plist)


def flat_grad_buffer(net, plist=None):
    """The persistent flat fp32 gradient buffer of ``net`` (registration order), created on demand."""
    plist = plist if plist is not None else list(net.parameters())
    total = sum(p.numel() for p in plist)
    buf = getattr(net, "_pmu_grad_flat", None)
    dev = plist[0].device
    if buf is None or buf.numel() != total or buf.device != dev:
        buf = torch.zeros(total, dtype=torch.float32, device=dev)
        net._pmu_grad_flat = buf
    return buf


def attach_flat_grad_views(net, plist):
    buf = flat_grad_buffer(net, plist)
    views, off = {}, 0
    for p in plist:
        n = p.numel()
        views[p] = buf[off:off + n].view_as(p)
        off += n
    net._pmu_grad_views = views


def unet_apply(net, x):
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise RuntimeError("UNet.forward runs on the MI355X HIP path only: move the model and input to the GPU "
                           "(there is no CPU fallback)")
    if x.dtype != torch.float32:
        x = x.float()
    params = list(net.parameters())
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return UNetFunction.apply(net, x, *params)
    with torch.no_grad():
        out, _ = engine.unet_forward(net, x, net.training)
    return out
