"""Standalone forward/backward of the drop-in blocks on the HIP engine (one autograd node per call).

``UNet.forward`` never calls these: it runs the whole stack as one fused node (engine.py), where a
layer's BatchNorm+ReLU, pooling, padding and concatenation are applied inside its consumer's
operand staging.  A block called on its own (as the reference's module tree allows) gets an
arbitrary NCHW tensor instead of a producer's pre-BN output, so here the input is a RAW operand
source and the block's output is materialised:

  DoubleConv   PMU/model/unet/unet_parts.py:9-24    conv3x3 -> BN -> ReLU, twice
  Down         unet_parts.py:27-38                  MaxPool2d(2) (pmu_frame_to_f32 on a pooled RAW
                                                    source; backward pmu_maxpool2_bwd, raw mode) + DoubleConv
  Up           unet_parts.py:41-67                  ConvTranspose2d(k2,s2) -> F.pad -> cat([skip, up])
                                                    (virtual: a two-source frame with offsets) -> DoubleConv
  OutConv      unet_parts.py:70-76                  1x1 conv (pmu_head1x1_fwd/_bwd, pmu_wgrad1x1)
  Encoder      probabilistic_unet.py:11-53          [AvgPool2d(2,ceil)] + (conv3x3 -> BN -> ReLU) x n per block

Outputs are NCHW-shaped views of channels-last (NHWC) storage, the engine's native layout.
Gradients follow the same flat-buffer / LiveNode rules as the fused nodes (functions.py).
"""
from __future__ import annotations

import torch

from . import _lib as L
from .engine import Src, _check_channels, _dc_layers, _empty, conv_bn_backward, conv_bn_forward, frame_of, pack_convT_weights
from .functions import LiveNode, _NO_CPU, grad_sink_for, use_bf16


def _nhwc(x: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor -> contiguous NHWC storage (free when it is channels-last already)."""
    t = x.detach().float().permute(0, 2, 3, 1)
    return t if t.is_contiguous() else t.contiguous()


def _check(name, *xs):
    for x in xs:
        if not isinstance(x, torch.Tensor) or not x.is_cuda or x.dim() != 4:
            raise RuntimeError(f"{name}.forward " + _NO_CPU)


def _act_out(o) -> torch.Tensor:
    """relu(bn(z)) of a ConvBNOut, materialised NHWC."""
    N, H, W, C = o.z.shape
    y = _empty(N, H, W, C, device=o.z.device)
    L.call("pmu_bnrelu_apply", o.z.data_ptr(), o.bn.coef.data_ptr(), N * H * W, C, y.data_ptr(), L.stream())
    return y


# ----------------------------------------------------------------------------------------
# runners: forward(inputs) -> (output NHWC, state); backward(state, dy NHWC, grads) -> [dx NHWC]
# ----------------------------------------------------------------------------------------
class _ConvStack:
    """A chain of (conv3x3, BN) layers, each consuming the previous one's BN+ReLU."""

    def __init__(self, layers, bf16):
        self.layers, self.bf16 = layers, bf16

    def forward(self, srcs, N, H, W, training, dev, planes=None, keep=True):
        outs = []
        for i, (conv, bn) in enumerate(self.layers):
            if i == 0:
                o = conv_bn_forward(srcs, conv, bn, N, H, W, training, dev, planes=planes, bf16=self.bf16, keep=keep)
            else:
                o = conv_bn_forward([outs[-1].act()], conv, bn, N, H, W, training, dev, bf16=self.bf16, keep=keep)
            outs.append(o)
        return outs

    def backward(self, outs, da, grads, need_dx=True, split=None):
        for i in reversed(range(len(self.layers))):
            conv, bn = self.layers[i]
            da = conv_bn_backward(outs[i], da, conv, bn, grads, need_dx=need_dx or i > 0,
                                  split=split if i == 0 else None)
            grads.flush()
        return da


def _first_srcs(xh, x_requires_grad):
    """Operand of a block's first conv: NCHW planes for the Cin <= 4 first-layer kernel when no
    input gradient is needed (it has no input-gradient pass), else the RAW NHWC tensor."""
    C = xh.shape[3]
    if C <= 4 and not x_requires_grad:
        return [], [xh[..., c].contiguous() for c in range(C)]
    return [Src(xh)], None


class DoubleConvRunner:
    def __init__(self, dc):
        self.module = dc
        c1, b1, c2, b2 = _dc_layers(dc)
        self.stack = _ConvStack([(c1, b1), (c2, b2)], use_bf16(dc))

    def forward(self, ins, training, keep=True):
        (x,), dev = ins, ins[0].device
        xh = _nhwc(x)
        N, H, W, _ = xh.shape
        srcs, planes = _first_srcs(xh, x.requires_grad)
        self.need_dx = planes is None
        outs = self.stack.forward(srcs, N, H, W, training, dev, planes=planes, keep=keep)
        return _act_out(outs[-1]), outs

    def backward(self, outs, dy, grads):
        dx = self.stack.backward(outs, dy, grads, need_dx=self.need_dx)
        return [dx]


class DownRunner:
    def __init__(self, down):
        self.module = down
        self.dc = DoubleConvRunner(down.maxpool_conv[1])

    def forward(self, ins, training, keep=True):
        (x,), dev = ins, ins[0].device
        xh = _nhwc(x)
        N, H, W, C = xh.shape
        if H < 2 or W < 2:
            raise RuntimeError("Down: MaxPool2d(2) needs H, W >= 2")
        h, w = H // 2, W // 2
        pooled = _empty(N, h, w, C, device=dev)
        L.call("pmu_frame_to_f32", frame_of([Src(xh, pool=L.POOL_MAX2)], N, h, w), pooled.data_ptr(), L.stream())
        outs = self.dc.stack.forward([Src(pooled)], N, h, w, training, dev, keep=keep)
        return _act_out(outs[-1]), (xh, outs)

    def backward(self, st, dy, grads):
        xh, outs = st
        dpool = self.dc.stack.backward(outs, dy, grads)
        N, H, W, C = xh.shape
        dx = _empty(N, H, W, C, device=xh.device)
        L.call("pmu_maxpool2_bwd", dpool.data_ptr(), xh.data_ptr(), None, N, H, W, C, dx.data_ptr(), 0, L.stream())
        return [dx]


class UpRunner:
    def __init__(self, up):
        self.module = up
        self.dc = DoubleConvRunner(up.conv)

    def forward(self, ins, training, keep=True):
        x1, x2 = ins
        dev = x1.device
        x1h, x2h = _nhwc(x1), _nhwc(x2)
        N, hi, wi, Cin = x1h.shape
        hs, ws_ = x2h.shape[1], x2h.shape[2]
        convT = self.module.up
        _check_channels(Cin, convT)
        Cup = convT.out_channels
        dY, dX = hs - 2 * hi, ws_ - 2 * wi
        if dY < 0 or dX < 0:
            raise RuntimeError("Up: the upsampled map is larger than the skip (F.pad would crop)")
        off = (dY // 2, dX // 2)
        u = _empty(N, 2 * hi, 2 * wi, Cup, device=dev)
        wpt = pack_convT_weights(convT.weight, dgrad=False)
        L.call("pmu_convT2x2_fwd", frame_of([Src(x1h)], N, hi, wi), convT.weight.data_ptr(), wpt.data_ptr(),
               L.ptr(convT.bias), Cup, u.data_ptr(), L.stream())
        srcs = [Src(x2h), Src(u, off=off)]
        outs = self.dc.stack.forward(srcs, N, hs, ws_, training, dev, keep=keep)
        return _act_out(outs[-1]), (x1h, x2h.shape[3], off, outs)

    def backward(self, st, dy, grads):
        x1h, Cskip, off, outs = st
        dskip, dup = self.dc.stack.backward(outs, dy, grads, split=Cskip)
        convT = self.module.up
        N, hi, wi, Cin = x1h.shape
        Hd, Wd, Cup = dup.shape[1], dup.shape[2], convT.out_channels
        s = L.stream()
        dx1 = _empty(N, hi, wi, Cin, device=x1h.device)
        wpt = pack_convT_weights(convT.weight, dgrad=True)
        L.call("pmu_convT2x2_dgrad", dup.data_ptr(), Hd, Wd, off[0], off[1], convT.weight.data_ptr(), wpt.data_ptr(),
               N, hi, wi, Cin, Cup, dx1.data_ptr(), s)
        dwt = grads.new(convT.weight)
        dbt = grads.new(convT.bias) if convT.bias is not None else None
        wsb = L.lib().pmu_convT2x2_wgrad_ws(N, hi, wi, Cin, Cup)
        ws = _empty(max(1, (wsb + 3) // 4), device=x1h.device)
        L.call("pmu_convT2x2_wgrad", dup.data_ptr(), Hd, Wd, off[0], off[1], frame_of([Src(x1h)], N, hi, wi), Cup,
               dwt.data_ptr(), L.ptr(dbt), ws.data_ptr(), wsb, s)
        grads.flush()
        return [dx1, dskip]


class OutConvRunner:
    def __init__(self, oc):
        self.module = oc

    def forward(self, ins, training, keep=True):
        (x,) = ins
        xh = _nhwc(x)
        N, H, W, C = xh.shape
        conv = self.module.conv
        K = conv.out_channels
        y = _empty(N, K, H, W, device=x.device)
        L.call("pmu_head1x1_fwd", frame_of([Src(xh)], N, H, W), conv.weight.data_ptr(), L.ptr(conv.bias), K, 0,
               y.data_ptr(), L.stream())
        return y.permute(0, 2, 3, 1), xh     # the NHWC view: _Block returns it NCHW-shaped

    def backward(self, xh, dy, grads):
        N, H, W, C = xh.shape
        conv = self.module.conv
        K = conv.out_channels
        s = L.stream()
        dyc = dy.permute(0, 3, 1, 2).contiguous()            # NCHW, as the head kernels take it
        dl = _empty(N, K, H, W, device=xh.device)
        da = _empty(N, H, W, C, device=xh.device)
        L.call("pmu_head1x1_bwd", dyc.data_ptr(), None, 0, conv.weight.data_ptr(), K, C, N, H, W, dl.data_ptr(),
               da.data_ptr(), s)
        dw = grads.new(conv.weight)
        db = grads.new(conv.bias) if conv.bias is not None else _empty(K, device=xh.device)
        wsb = L.lib().pmu_wgrad1x1_ws(N * H * W, K, C)
        ws = _empty(max(1, (wsb + 3) // 4), device=xh.device)
        L.call("pmu_wgrad1x1", dl.data_ptr(), frame_of([Src(xh)], N, H, W), K, dw.data_ptr(), db.data_ptr(),
               ws.data_ptr(), wsb, s)
        grads.flush()
        return [da]


class EncoderRunner:
    """Encoder.forward (probabilistic_unet.py:51-53) alone: the encoder layers with AvgPool2d(2, ceil)
    fused into the next conv's staging; the last BN+ReLU materialised."""

    def __init__(self, enc):
        from .prob_engine import encoder_layers
        self.module = enc
        self.layers = encoder_layers(enc)

    def forward(self, ins, training, keep=True):
        (x,), dev = ins, ins[0].device
        xh = _nhwc(x)
        N, H, W, _ = xh.shape
        srcs, planes = _first_srcs(xh, x.requires_grad)
        self.need_dx = planes is None
        if self.layers[0][2]:
            raise NotImplementedError("encoder first layer: no pooling")
        outs, h, w = [], H, W
        for idx, (conv, bn, pooled) in enumerate(self.layers):
            if idx == 0:
                o = conv_bn_forward(srcs, conv, bn, N, H, W, training, dev, planes=planes, keep=keep)
            else:
                if pooled:
                    h, w = (h + 1) // 2, (w + 1) // 2
                o = conv_bn_forward([outs[-1].act(L.POOL_AVG2CEIL if pooled else L.POOL_NONE)], conv, bn, N, h, w,
                                    training, dev, keep=keep)
            outs.append(o)
        return _act_out(outs[-1]), outs

    def backward(self, outs, da, grads):
        s = L.stream()
        for idx in reversed(range(len(self.layers))):
            conv, bn, pooled = self.layers[idx]
            dx = conv_bn_backward(outs[idx], da, conv, bn, grads, need_dx=idx > 0 or self.need_dx)
            grads.flush()
            if idx == 0:
                return [dx]
            if pooled:
                p = outs[idx - 1].z
                N, hp, wp, Cp = p.shape
                da = _empty(N, hp, wp, Cp, device=p.device)
                L.call("pmu_avgpool2_bwd", dx.data_ptr(), N, hp, wp, Cp, da.data_ptr(), s)
            else:
                da = dx


# ----------------------------------------------------------------------------------------
# autograd node
# ----------------------------------------------------------------------------------------
class _Block(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, n_in, *args):
        ins = args[:n_in]
        out, st = runner.forward(ins, runner.module.training, keep=True)
        ctx.runner, ctx.st, ctx.n_in = runner, st, n_in
        ctx.live = LiveNode(runner.module)
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        r = ctx.runner
        plist = list(r.module.parameters())
        sink = grad_sink_for(r.module, plist)
        ctx.live.release()
        dins = r.backward(ctx.st, _nhwc(dy), sink)
        sink.flush()
        ctx.st = None
        dins = [d.permute(0, 3, 1, 2) if d is not None else None for d in dins]
        return (None, None) + tuple(dins) + tuple(sink.get(p) for p in plist)


def _apply(runner, name, *xs):
    _check(name, *xs)
    params = list(runner.module.parameters())
    if torch.is_grad_enabled() and (any(p.requires_grad for p in params) or any(x.requires_grad for x in xs)):
        return _Block.apply(runner, len(xs), *xs, *params)
    with torch.no_grad():
        out, _ = runner.forward(xs, runner.module.training, keep=False)
    return out.permute(0, 3, 1, 2)


def double_conv_apply(dc, x):
    return _apply(DoubleConvRunner(dc), "DoubleConv", x)


def down_apply(down, x):
    return _apply(DownRunner(down), "Down", x)


def up_apply(up, x1, x2):
    return _apply(UpRunner(up), "Up", x1, x2)


def outconv_apply(oc, x):
    return _apply(OutConvRunner(oc), "OutConv", x)


def encoder_apply(enc, x):
    return _apply(EncoderRunner(enc), "Encoder", x)
