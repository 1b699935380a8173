"""Forward/backward executor of the Probabilistic U-Net's own parts on libpmunet_hip (rows a9-a11).

  AxisAlignedConvGaussian (encoder + spatial mean + 1x1 latent head)
        PMU/model/probabilistic_unet/probabilistic_unet.py:11-114
  Fcomb (1x1 chain on cat(features, tile(z)))     probabilistic_unet.py:116-181

The encoder reuses the U-Net conv/BN executor (engine.conv_bn_forward/backward): AvgPool2d(2,
ceil) is fused into the next conv's operand staging (PMU_POOL_AVG2CEIL), BN+ReLU into the
consumer, exactly as MaxPool2d is for the U-Net.  The 1x1 latent conv on the 1x1 mean map is a
tiny (N x C) . (C x 2L) product.  Fcomb never materialises the tiled z: W_1 . [f; z] =
W_1f . f + (W_1z . z + b_1), the bracket being a per-(sample, image) bias.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import _lib as L
from .engine import ConvBNOut, _empty, conv_bn_backward, conv_bn_forward

F32 = torch.float32


# ----------------------------------------------------------------------------------------
# encoder + latent head
# ----------------------------------------------------------------------------------------
def encoder_layers(enc):
    """[(conv, bn, pooled_before)] of an Encoder's Sequential (probabilistic_unet.py:26-47),
    validated against what the HIP path implements."""
    mods = list(enc.layers)
    out, pooled = [], False
    for i, m in enumerate(mods):
        if isinstance(m, nn.AvgPool2d):
            if not (m.kernel_size in (2, (2, 2)) and m.stride in (2, (2, 2)) and m.padding in (0, (0, 0))
                    and m.ceil_mode):
                raise NotImplementedError("Encoder pooling other than AvgPool2d(2, 2, 0, ceil_mode=True)")
            pooled = True
        elif isinstance(m, nn.Conv2d):
            bn = mods[i + 1] if i + 1 < len(mods) else None
            if m.kernel_size != (3, 3) or m.padding != (1, 1) or m.stride != (1, 1) or not isinstance(bn, nn.BatchNorm2d):
                raise NotImplementedError("Encoder layers other than Conv2d(3x3, pad 1) + BatchNorm2d")
            out.append((m, bn, pooled))
            pooled = False
    return out


@dataclass
class GaussState:
    layers: list          # ConvBNOut per conv
    mean: torch.Tensor    # (N, C) spatial mean of the last activation
    hw: tuple


def gaussian_forward(g, planes, training: bool, keep: bool = False):
    """AxisAlignedConvGaussian.forward up to mu_log_sigma (N, 2L) (probabilistic_unet.py:82-105).
    ``planes``: the input channels (cat(input, segm) for the posterior) as contiguous (N,H,W) maps.
    keep: a backward follows (the convs keep their operand copies for the weight gradients)."""
    dev = planes[0].device
    N, H, W = planes[0].shape
    layers = encoder_layers(g.encoder)
    outs = []
    h, w = H, W
    prev: ConvBNOut | None = None
    for idx, (conv, bn, pooled) in enumerate(layers):
        if idx == 0:
            if len(planes) > 4 or pooled:
                raise NotImplementedError("encoder first layer: at most 4 input channels, no pooling")
            o = conv_bn_forward([], conv, bn, N, H, W, training, dev, planes=planes)
        else:
            if pooled:
                h, w = (h + 1) // 2, (w + 1) // 2
            o = conv_bn_forward([prev.act(L.POOL_AVG2CEIL if pooled else L.POOL_NONE)], conv, bn, N, h, w,
                                training, dev, keep=keep)
        outs.append(o)
        prev = o
    C = prev.z.shape[3]
    s = L.stream()
    mean = _empty(N, C, device=dev)
    L.call("pmu_spatial_mean", prev.z.data_ptr(), prev.bn.coef.data_ptr(), N, h, w, C, mean.data_ptr(), s)
    cl = g.conv_layer
    M = cl.out_channels
    if cl.kernel_size != (1, 1) or cl.in_channels != C:
        raise NotImplementedError("latent head must be a 1x1 conv on the encoder output")
    mls = _empty(N, M, device=dev)
    L.call("pmu_linear_fwd", mean.data_ptr(), cl.weight.data_ptr(), L.ptr(cl.bias), N, C, M, mls.data_ptr(), s)
    return mls, GaussState(layers=outs, mean=mean, hw=(h, w))


def gaussian_backward(g, st: GaussState, dmls: torch.Tensor, grads):
    """Backward of gaussian_forward given dL/d(mu_log_sigma); parameter grads go to ``grads``."""
    s = L.stream()
    dev = dmls.device
    layers = encoder_layers(g.encoder)
    N, C = st.mean.shape
    cl = g.conv_layer
    M = cl.out_channels
    dmls = dmls.contiguous()
    dmean = _empty(N, C, device=dev)
    dwl = grads.new(cl.weight)
    dbl = grads.new(cl.bias) if cl.bias is not None else None
    L.call("pmu_linear_bwd", st.mean.data_ptr(), cl.weight.data_ptr(), dmls.data_ptr(), N, C, M, dmean.data_ptr(),
           dwl.data_ptr(), L.ptr(dbl), s)
    h, w = st.hw
    da = _empty(N, h, w, C, device=dev)
    lb = L.lib()

    def fused(o):   # the pass that completes o's da can form o's BN-backward partial sums (fp32 z, C % 4)
        return o.z.dtype == torch.float32 and o.bn.mean is not None and o.z.shape[3] % 4 == 0

    def bnr_call(name, g, o, da):
        Np, hp, wp, Cp = o.z.shape
        R = lb.pmu_bn_bwd_tiles(Np * hp * wp, Cp)
        part = _empty(R, 2 * Cp, device=dev)
        L.call(name, g.data_ptr(), o.z.data_ptr(), o.bn.coef.data_ptr(), o.bn.mean.data_ptr(),
               o.bn.invstd.data_ptr(), Np, hp, wp, Cp, da.data_ptr(), part.data_ptr(), s)
        o.bnr = (da, part, R)

    last = st.layers[-1]
    if fused(last):
        bnr_call("pmu_spatial_mean_bwd_bnr", dmean, last, da)
    else:
        L.call("pmu_spatial_mean_bwd", dmean.data_ptr(), N, h, w, C, da.data_ptr(), s)
    for idx in reversed(range(len(layers))):
        conv, bn, pooled = layers[idx]
        o = st.layers[idx]
        dx = conv_bn_backward(o, da, conv, bn, grads, need_dx=(idx > 0))
        if idx == 0:
            break
        if pooled:
            prev = st.layers[idx - 1]
            hp, wp, Cp = prev.z.shape[1], prev.z.shape[2], prev.z.shape[3]
            da = _empty(N, hp, wp, Cp, device=dev)
            if fused(prev):
                # the pooled layer's da is complete here: its BN-backward partials in the same pass
                bnr_call("pmu_avgpool2_bwd_bnr", dx, prev, da)
            else:
                L.call("pmu_avgpool2_bwd", dx.data_ptr(), N, hp, wp, Cp, da.data_ptr(), s)
        else:
            da = dx
    return grads


# ----------------------------------------------------------------------------------------
# Fcomb
# ----------------------------------------------------------------------------------------
def fcomb_layers(fc):
    """(hidden 1x1 convs, last 1x1 conv) of an Fcomb, validated for the fused kernels."""
    convs = [m for m in fc.layers if isinstance(m, nn.Conv2d)]
    acts = [m for m in fc.layers if not isinstance(m, nn.Conv2d)]
    last = fc.last_layer
    F_ = convs[0].out_channels
    ok = (1 <= len(convs) <= 3 and all(isinstance(a, nn.ReLU) for a in acts) and len(acts) == len(convs)
          and F_ <= 64 and last.out_channels <= 32 and last.in_channels == F_
          and all(c.kernel_size == (1, 1) and c.bias is not None for c in convs + [last])
          and all(c.in_channels == F_ and c.out_channels == F_ for c in convs[1:]))
    if not ok:
        raise NotImplementedError("Fcomb shape outside the fused kernel's range "
                                  "(<= 3 hidden 1x1 convs of width <= 64, <= 32 classes)")
    return convs, last


def _ptr_array(ts):
    return (ctypes.c_void_p * 3)(*([t.data_ptr() for t in ts] + [None] * (3 - len(ts))))


def features_nhwc(feat: torch.Tensor) -> torch.Tensor:
    """(N,F,H,W) feature map -> contiguous NHWC storage (free for the U-Net's channels-last output)."""
    f = feat.permute(0, 2, 3, 1)
    return f if f.is_contiguous() else f.contiguous()


def fcomb_forward(fc, feat: torch.Tensor, z: torch.Tensor):
    """logits for S samples: feat (N,F,H,W), z (S,N,L) -> (S,N,K,H,W), plus zb for backward."""
    convs, last = fcomb_layers(fc)
    fh = features_nhwc(feat)
    N, H, W, F_ = fh.shape
    S, Nz, Lz = z.shape
    if Nz != N or convs[0].in_channels != F_ + Lz:
        raise RuntimeError(f"Fcomb: features {tuple(feat.shape)} and z {tuple(z.shape)} do not concatenate "
                           f"to the {convs[0].in_channels} input channels of the first 1x1 conv")
    K = last.out_channels
    dev = feat.device
    s = L.stream()
    zc = z.contiguous().float()
    zb = _empty(S * N, F_, device=dev)
    L.call("pmu_fcomb_zbias", zc.data_ptr(), convs[0].weight.data_ptr(), convs[0].bias.data_ptr(), S * N, F_, Lz,
           zb.data_ptr(), s)
    y = _empty(S, N, K, H, W, device=dev)
    L.call("pmu_fcomb_fwd", fh.data_ptr(), zb.data_ptr(), _ptr_array([c.weight for c in convs]),
           _ptr_array([c.bias for c in convs]), last.weight.data_ptr(), last.bias.data_ptr(), F_, Lz, K, len(convs),
           S, N, H, W, y.data_ptr(), s)
    return y, fh, zc, zb


def fcomb_backward(fc, fh, zc, zb, dy: torch.Tensor, grads):
    """One sample: dy = dL/dlogits (N,K,H,W) -> (dfeat NHWC, dz (N,L)); parameter grads to ``grads``."""
    convs, last = fcomb_layers(fc)
    N, H, W, F_ = fh.shape
    Lz = zc.shape[-1]
    K = last.out_channels
    dev = fh.device
    s = L.stream()
    dyc = dy.contiguous()
    dfeat = _empty(N, H, W, F_, device=dev)
    dz = _empty(N, Lz, device=dev)
    dws = [grads.new(c.weight) for c in convs]
    dbs = [grads.new(c.bias) for c in convs]
    dwl, dbl = grads.new(last.weight), grads.new(last.bias)
    wsb = L.lib().pmu_fcomb_bwd_ws(N, H, W)
    ws = _empty(max(1, (wsb + 3) // 4), device=dev)
    L.call("pmu_fcomb_bwd", fh.data_ptr(), zc.data_ptr(), zb.data_ptr(), dyc.data_ptr(),
           _ptr_array([c.weight for c in convs]), _ptr_array([c.bias for c in convs]), last.weight.data_ptr(),
           last.bias.data_ptr(), F_, Lz, K, len(convs), N, H, W, dfeat.data_ptr(), dz.data_ptr(),
           _ptr_array(dws), _ptr_array(dbs), dwl.data_ptr(), dbl.data_ptr(), ws.data_ptr(), wsb, s)
    return dfeat, dz
