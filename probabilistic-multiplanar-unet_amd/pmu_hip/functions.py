"""Autograd bridge: one torch.autograd.Function per fused network part, backed by the HIP executors.

The reference builds one autograd node per PyTorch op (~90 for the 5-level U-Net); here the
whole U-Net forward is a single node whose backward replays the stack in reverse on the HIP
kernels and returns every parameter gradient at once.  The Probabilistic U-Net adds two more
node kinds: the prior/posterior AxisAlignedConvGaussian (encoder + latent head) and Fcomb.

Gradients: when every ``.grad`` of a node's parameters is None (zero_grad(set_to_none=True)),
the kernels write straight into fresh views of one persistent flat buffer owned by the root
module (the U-Net, or the ProbabilisticUnet that contains it); autograd adopts those views as
``.grad``, so all gradients are contiguous for one all-reduce and pointer-stable for FusedSGD.
"""
from __future__ import annotations

import weakref

import torch

from . import engine, prob_engine
from .engine import GradSink

_NO_CPU = "runs on the MI355X HIP path only: move the model and inputs to the GPU (there is no CPU fallback)"


# ----------------------------------------------------------------------------------------
# flat gradient buffer
# ----------------------------------------------------------------------------------------
def set_grad_root(module, root):
    """Make ``module``'s gradient views live in ``root``'s flat buffer (not a submodule link)."""
    module.__dict__["_pmu_root_ref"] = weakref.ref(root)


def grad_root(module):
    ref = module.__dict__.get("_pmu_root_ref")
    root = ref() if ref is not None else None
    return root if root is not None else module


ALIGN = 64   # every slot starts on a 256-B boundary: the fused optimizer streams float4


def _slot(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def grad_layout(net, plist):
    """Parameters in flat-buffer order: the order the backward produced them when one was recorded
    (``set_grad_order``, pmu_hip.dp learns it from the first step), else registration order."""
    order = net.__dict__.get("_pmu_grad_order")
    if order is None:
        return list(plist)
    pos = {pid: i for i, pid in enumerate(order)}
    return sorted(plist, key=lambda p: pos.get(id(p), len(pos)))


def set_grad_order(net, params_in_order):
    """Lay the flat gradient buffer out in this parameter order from the next backward on (the
    current .grad views keep the old layout until they are released)."""
    net.__dict__["_pmu_grad_order"] = [id(p) for p in params_in_order]
    net.__dict__["_pmu_grad_offsets"] = None


def flat_grad_buffer(net, plist=None):
    """The persistent flat fp32 gradient buffer of ``net``, created on demand: one 64-float aligned
    slot per parameter (pads stay zero), in ``grad_layout`` order."""
    plist = plist if plist is not None else list(net.parameters())
    total = sum(_slot(p.numel()) for p in plist)
    buf = net.__dict__.get("_pmu_grad_flat")
    dev = plist[0].device
    if buf is None or buf.numel() != total or buf.device != dev:
        buf = torch.zeros(total, dtype=torch.float32, device=dev)
        net.__dict__["_pmu_grad_flat"] = buf
        net.__dict__["_pmu_grad_offsets"] = None
    return buf


def _offsets(root, plist):
    """{id(param): element offset of its slot in the flat buffer}."""
    cached = root.__dict__.get("_pmu_grad_offsets")
    key = tuple(id(p) for p in plist)
    if cached is None or cached[0] != key:
        offs, o = {}, 0
        for p in grad_layout(root, plist):
            offs[id(p)] = o
            o += _slot(p.numel())
        cached = (key, offs)
        root.__dict__["_pmu_grad_offsets"] = cached
    return cached[1]


class LiveNode:
    """Marks one pending autograd node of ``module`` (created in forward, released when its backward
    has run or its graph was freed); ``module._pmu_live`` counts them (diagnostics and tests)."""
    __slots__ = ("d",)

    def __init__(self, module):
        self.d = module.__dict__
        self.d["_pmu_live"] = self.d.get("_pmu_live", 0) + 1

    def release(self):
        if self.d is not None:
            self.d["_pmu_live"] -= 1
            self.d = None

    def __del__(self):
        self.release()


def grad_sink_for(module, params) -> GradSink:
    """Destination of this node's parameter gradients (fresh flat-buffer views, see module doc).
    The views are created per backward and not retained, so autograd can adopt them as .grad.

    Plain tensors instead when a .grad already exists (autograd accumulates into it), or when
    another node of the same module already received the views in this same backward pass (the
    module applied twice in one graph, e.g. loss(net(x1)) + loss(net(x2))): autograd sums the two
    node outputs before AccumulateGrad, and aliased views would give 2*g2 instead of g1 + g2.  A
    second node that is pending but never reached by the backward (the Probabilistic U-Net's prior
    sample ``masks_pred``, alive while -elbo backpropagates) does not count: the test is per
    autograd graph task, not per pending node.

    Either way the sink reports its layers to the root's data-parallel reducer (``on_ready``), so
    the backward order is learned even from a step whose last backward accumulates into existing
    .grad tensors (several micro-batches per rank); only flat-buffer sinks let it issue buckets."""
    root = grad_root(module)
    ready = root.__dict__.get("_pmu_grad_ready")
    task = torch._C._current_graph_task_id()
    d = module.__dict__
    if not all(p.grad is None for p in params) or (task >= 0 and d.get("_pmu_views_task") == task):
        return GradSink(on_ready=ready)
    d["_pmu_views_task"] = task
    plist = list(root.parameters())
    buf = flat_grad_buffer(root, plist)
    offs = _offsets(root, plist)
    views = {}
    for p in params:
        o = offs.get(id(p))
        if o is not None:
            views[p] = buf[o:o + p.numel()].view_as(p)
    return GradSink(views, on_ready=ready)


# ----------------------------------------------------------------------------------------
# independent network parts on concurrent HIP streams
# ----------------------------------------------------------------------------------------
_SIDE_STREAMS: dict = {}


def _side_stream(dev, i):
    key = (dev.index, i)
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return s


def _record(obj, stream):
    """Mark every tensor reachable from a part's result (tensors, distributions' loc/scale, tuples)
    as used on ``stream``, so the caching allocator does not hand its memory back to the producing side
    stream while ``stream`` may still read it."""
    if isinstance(obj, torch.Tensor):
        obj.record_stream(stream)
    elif isinstance(obj, (tuple, list)):
        for o in obj:
            _record(o, stream)
    elif hasattr(obj, "base_dist"):
        _record(obj.base_dist, stream)
    elif hasattr(obj, "loc") and hasattr(obj, "scale"):
        _record((obj.loc, obj.scale), stream)


def run_concurrent(dev, parts):
    """Run independent network parts (callables) with part 0 on the current stream and part i on side
    stream i, each side stream starting behind everything already queued on the current one; the current
    stream then waits for all of them.  The HIP executors launch on torch's current stream
    (pmu_hip._lib.stream), so a part's kernels — and, through autograd's stream semantics, its backward,
    which runs on the stream of its forward — overlap the other parts'.  Used by the Probabilistic U-Net's
    forward for its UNet, prior and posterior (PMU/model/probabilistic_unet/probabilistic_unet.py:215-223),
    whose deep 32^2 / 16^2 layers alone do not fill the chip.  Returns the parts' results in order."""
    main = torch.cuda.current_stream(dev)
    res = [None] * len(parts)
    sides = []
    for i in range(1, len(parts)):
        s = _side_stream(dev, i)
        s.wait_stream(main)
        with torch.cuda.stream(s):
            res[i] = parts[i]()
        sides.append((i, s))
    res[0] = parts[0]()
    for i, s in sides:
        main.wait_stream(s)
        _record(res[i], main)
    return res


# ----------------------------------------------------------------------------------------
# U-Net
# ----------------------------------------------------------------------------------------
def use_bf16(net) -> bool:
    """bf16-MFMA arithmetic for this call: inside torch.autocast("cuda", dtype=torch.bfloat16) —
    the PyTorch idiom for the reference's config c5 — or when ``net.pmu_precision == "bf16"``."""
    if getattr(net, "pmu_precision", None) == "bf16":
        return True
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


class UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net, x, bf16, *params):
        out, st = engine.unet_forward(net, x, net.training, bf16=bf16, keep=True)
        ctx.net = net
        ctx.st = st
        ctx.live = LiveNode(net)
        return out

    @staticmethod
    def backward(ctx, dy):
        net = ctx.net
        plist = list(net.parameters())
        sink = grad_sink_for(net, plist)
        ctx.live.release()
        grads = engine.unet_backward(net, ctx.st, dy, sink)
        grads.flush()
        ctx.st = None
        return (None, None, None) + tuple(grads.get(p) for p in plist)


def unet_apply(net, x):
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise RuntimeError("UNet.forward " + _NO_CPU)
    if x.dtype != torch.float32:
        x = x.float()
    params = list(net.parameters())
    bf16 = use_bf16(net)
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return UNetFunction.apply(net, x, bf16, *params)
    with torch.no_grad():
        out, _ = engine.unet_forward(net, x, net.training, bf16=bf16)
    return out


# ----------------------------------------------------------------------------------------
# AxisAlignedConvGaussian: input planes -> mu_log_sigma (N, 2L)
# ----------------------------------------------------------------------------------------
def _planes(x, segm):
    ps = [x[:, c] for c in range(x.shape[1])]
    if segm is not None:
        ps += [segm[:, c] for c in range(segm.shape[1])]
    return [p.contiguous().float() for p in ps]


class GaussianFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, x, segm, *params):
        mls, st = prob_engine.gaussian_forward(g, _planes(x, segm), g.training, keep=True)
        g.__dict__["_pmu_enc_out"] = (st.layers[-1].z, st.layers[-1].bn.coef)
        ctx.g, ctx.st = g, st
        ctx.live = LiveNode(g)
        return mls

    @staticmethod
    def backward(ctx, dmls):
        g = ctx.g
        plist = list(g.parameters())
        sink = grad_sink_for(g, plist)
        ctx.live.release()
        grads = prob_engine.gaussian_backward(g, ctx.st, dmls, sink)
        grads.flush()
        ctx.st = None
        return (None, None, None) + tuple(grads.get(p) for p in plist)


def gaussian_apply(g, x, segm=None):
    """mu_log_sigma (N, 2L) of AxisAlignedConvGaussian.forward (probabilistic_unet.py:82-105)."""
    for t in (x, segm):
        if t is not None and (not isinstance(t, torch.Tensor) or not t.is_cuda):
            raise RuntimeError("AxisAlignedConvGaussian.forward " + _NO_CPU)
    params = list(g.parameters())
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return GaussianFunction.apply(g, x, segm, *params)
    with torch.no_grad():
        mls, st = prob_engine.gaussian_forward(g, _planes(x, segm), g.training)
    g.__dict__["_pmu_enc_out"] = (st.layers[-1].z, st.layers[-1].bn.coef)
    return mls


def gaussian_encoding(g):
    """The last forward's encoder output relu(bn(z)) as an NCHW-shaped (channels-last) tensor, or 0."""
    zc = g.__dict__.get("_pmu_enc_out")
    if zc is None:
        return 0
    from . import _lib as L
    z, coef = zc
    N, H, W, C = z.shape
    out = torch.empty_like(z)
    L.call("pmu_bnrelu_apply", z.data_ptr(), coef.data_ptr(), N * H * W, C, out.data_ptr(), L.stream())
    return out.permute(0, 3, 1, 2)


def encoder_apply(enc, x):
    """Encoder.forward called on its own (probabilistic_unet.py:51-53)."""
    from .blocks import encoder_apply as _enc
    return _enc(enc, x)


# ----------------------------------------------------------------------------------------
# Fcomb: (features, z) -> logits
# ----------------------------------------------------------------------------------------
class FcombFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fc, feat, z, *params):
        y, fh, zc, zb = prob_engine.fcomb_forward(fc, feat, z.unsqueeze(0))
        ctx.fc = fc
        ctx.save = (fh, zc[0], zb)
        ctx.live = LiveNode(fc)
        return y[0]

    @staticmethod
    def backward(ctx, dy):
        fc = ctx.fc
        fh, zc, zb = ctx.save
        plist = list(fc.parameters())
        grads = grad_sink_for(fc, plist)
        ctx.live.release()
        dfeat, dz = prob_engine.fcomb_backward(fc, fh, zc, zb, dy, grads)
        grads.flush()
        ctx.save = None
        # dfeat is NHWC storage; hand it back with the (N,F,H,W) shape of the features input
        return (None, dfeat.permute(0, 3, 1, 2), dz) + tuple(grads.get(p) for p in plist)


def fcomb_apply(fc, feat, z):
    """Fcomb.forward (probabilistic_unet.py:167-181): feat (N,F,H,W), z (N,L) -> logits (N,K,H,W)."""
    for t in (feat, z):
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise RuntimeError("Fcomb.forward " + _NO_CPU)
    params = list(fc.parameters())
    needs = torch.is_grad_enabled() and (feat.requires_grad or z.requires_grad or any(p.requires_grad for p in params))
    if needs:
        return FcombFunction.apply(fc, feat, z, *params)
    with torch.no_grad():
        y, _, _, _ = prob_engine.fcomb_forward(fc, feat, z.unsqueeze(0))
    return y[0]


def fcomb_samples(fc, feat, zs):
    """S samples in one pass (features read once): zs (S,N,L) -> (S,N,K,H,W).  No autograd."""
    if not feat.is_cuda or not zs.is_cuda:
        raise RuntimeError("Fcomb sampling " + _NO_CPU)
    with torch.no_grad():
        y, _, _, _ = prob_engine.fcomb_forward(fc, feat, zs)
    return y
