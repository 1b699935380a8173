"""Forward/backward executor of the U-Net conv stack on libpmunet_hip.

Everything here only enqueues HIP kernels on the current torch stream through the C ABI;
PyTorch supplies device memory (caching allocator) and the stream.  Activations live
channels-last (NHWC) between kernels; a layer's output is kept as its *pre-BN* conv result
``z`` plus per-channel BN coefficients, and the consumer applies BN+ReLU (+pool / +concat)
while staging its operand, so post-activation tensors are never materialised.

Reference call graph mirrored here (PMU/ = Probabilistic-Multiplanar-Unet/):
  UNet.forward                 PMU/model/unet/unet_model.py:31-54
  DoubleConv / Down / Up / OutConv   PMU/model/unet/unet_parts.py:9-76
"""
from __future__ import annotations

import ctypes
import os
import weakref
from dataclasses import dataclass, field

import torch

from . import _lib as L

F32 = torch.float32
BF16S = torch.int16   # bf16 values kept as their 16-bit patterns (the kernels' unsigned short)


# ----------------------------------------------------------------------------------------
# operand descriptors
# ----------------------------------------------------------------------------------------
@dataclass
class Src:
    """One channel source of a conv operand (see pmu_src in include/pmunet_hip.h)."""
    x: torch.Tensor                  # NHWC [N][H][W][C]
    mode: int = L.SRC_RAW
    coef: torch.Tensor | None = None
    z: torch.Tensor | None = None    # BNBWD only
    pool: int = L.POOL_NONE
    off: tuple = (0, 0)
    prod: object = None              # the ConvBNOut whose activation this is (SRC_BNRELU sources)

    @property
    def C(self) -> int:
        return self.x.shape[3]

    def frame_hw(self):
        H, W = self.x.shape[1], self.x.shape[2]
        if self.pool == L.POOL_MAX2:
            return H // 2, W // 2
        if self.pool == L.POOL_AVG2CEIL:
            return (H + 1) // 2, (W + 1) // 2
        return H, W


def make_frame(srcs, N: int, H: int, W: int) -> L.PmuFrame:
    f = L.PmuFrame()
    f.nsrc = len(srcs)
    f.N, f.H, f.W = N, H, W
    for i, s in enumerate(srcs):
        t = s.x
        assert t.is_contiguous() and t.dtype in (F32, BF16S) and t.dim() == 4, \
            "operand must be contiguous NHWC fp32 (or bf16 bits)"
        c = f.src[i]
        c.x = t.data_ptr()
        c.z = s.z.data_ptr() if s.z is not None else None
        c.dtype = (L.DT_X_BF16 if t.dtype == BF16S else 0) | (L.DT_Z_BF16 if s.z is not None and s.z.dtype == BF16S else 0)
        c.coef = s.coef.data_ptr() if s.coef is not None else None
        c.mode, c.pool = s.mode, s.pool
        c.C, c.H, c.W = t.shape[3], t.shape[1], t.shape[2]
        c.off_h, c.off_w = s.off
    return f


def frame_of(srcs, N, H, W):
    return ctypes.byref(make_frame(srcs, N, H, W))


def _f32_srcs(srcs, N, H, W):
    """srcs for a call that stages fp32 frames itself (the fused-staging kernels): unchanged when every
    source is stored in fp32, else the frame's values materialised once in fp32 as one RAW source."""
    if all(sr.x.dtype == F32 and (sr.z is None or sr.z.dtype == F32) for sr in srcs):
        return srcs
    return [Src(frame_to_f32(srcs, N, H, W))]


def _materialised(srcs, dtype):
    """The operand tensor itself when the frame is one RAW, unpooled, unshifted source already stored
    in the dtype the GEMM reads (fp32, or bf16 with channels padded to 8): no copy is needed."""
    if len(srcs) != 1:
        return None
    sr = srcs[0]
    if (sr.mode != L.SRC_RAW or sr.pool != L.POOL_NONE or sr.off != (0, 0) or sr.x.dtype != dtype
            or not sr.x.is_contiguous() or sr.x.dim() != 4):
        return None
    if dtype == BF16S and sr.C % 8 != 0:
        return None
    return sr.x


def _empty(*shape, dtype=F32, device=None):
    return torch.empty(shape, dtype=dtype, device=device)


class GradSink(dict):
    """param -> gradient tensor.  ``new(p)`` hands out the destination a kernel writes: a view
    of the network's persistent flat gradient buffer when one is attached (stable pointers for
    the fused optimizer / one-shot all-reduce), else a fresh tensor.

    ``on_ready``: called by ``flush()`` as ``on_ready(params, flat)`` with the parameters whose
    gradient kernels have been enqueued on the stream since the previous flush, so a
    data-parallel reducer (pmu_hip.dp) can learn the backward order and, for a flat-buffer sink
    (``flat``), start a bucket's all-reduce while the rest of the backward still runs."""

    def __init__(self, views=None, on_ready=None):
        super().__init__()
        self.views = views
        self.flat = views is not None
        self.on_ready = on_ready
        self._pending = []

    def new(self, p):
        t = self.views.get(p) if self.views is not None else None
        if t is None:
            t = torch.empty_like(p)
        self[p] = t
        if self.on_ready is not None:
            self._pending.append(p)
        return t

    def flush(self):
        if self.on_ready is not None and self._pending:
            ready, self._pending = self._pending, []
            self.on_ready(ready, self.flat)


# ----------------------------------------------------------------------------------------
# BatchNorm
# ----------------------------------------------------------------------------------------
@dataclass
class BNState:
    coef: torch.Tensor      # [scale | shift]
    mean: torch.Tensor | None = None
    invstd: torch.Tensor | None = None
    count: float = 0.0


def bn_forward(part, R: int, C: int, count: int, bn: torch.nn.BatchNorm2d, training: bool, dev) -> BNState:
    """BatchNorm2d statistics (train) or running-stat coefficients (eval)."""
    s = L.stream()
    use_batch = training or not bn.track_running_stats or bn.running_mean is None
    if not use_batch:
        coef = _empty(2 * C, device=dev)
        L.call("pmu_bn_eval_coef", bn.running_mean.data_ptr(), bn.running_var.data_ptr(), L.ptr(bn.weight),
               L.ptr(bn.bias), float(bn.eps), C, coef.data_ptr(), s)
        return BNState(coef=coef)
    G = L.lib().pmu_colsum_groups(R)
    acc = _empty(G, 2 * C, dtype=torch.float64, device=dev)
    L.call("pmu_colsum_f64", part.data_ptr(), R, 2 * C, acc.data_ptr(), G, s)
    mean, invstd, coef = _empty(C, device=dev), _empty(C, device=dev), _empty(2 * C, device=dev)
    update = training and bn.track_running_stats and bn.running_mean is not None
    momentum = bn.momentum
    nbt = None  # the finalize kernel adds 1 to num_batches_tracked (one launch fewer per layer)
    if update:
        if momentum is None:  # cumulative moving average: the host needs the count now
            bn.num_batches_tracked.add_(1)
            momentum = 1.0 / float(bn.num_batches_tracked.item())
        elif bn.num_batches_tracked.dtype == torch.int64 and bn.num_batches_tracked.device == dev:
            nbt = bn.num_batches_tracked.data_ptr()
        else:
            bn.num_batches_tracked.add_(1)
    L.call("pmu_bn_fwd_finalize", acc.data_ptr(), G, C, float(count), L.ptr(bn.weight), L.ptr(bn.bias),
           float(bn.eps), float(momentum or 0.0),
           bn.running_mean.data_ptr() if update else None, bn.running_var.data_ptr() if update else None,
           nbt, mean.data_ptr(), invstd.data_ptr(), coef.data_ptr(), s)
    return BNState(coef=coef, mean=mean, invstd=invstd, count=float(count))


def bn_backward(da: torch.Tensor, z: torch.Tensor, st: BNState, bn: torch.nn.BatchNorm2d, grads, conv_bias=None,
                pre=None):
    """Returns (bcoef, dgamma, dbeta, dbias) for BN+ReLU backward given da = dL/d relu(bn(z)).
    pre: (part, R) — the partial sums (sum g, sum g*xhat) already formed by the kernel that produced
    da (a *_bnr input gradient); else pmu_bn_bwd_reduce reads da and z for them."""
    s = L.stream()
    dev = z.device
    N, H, W, C = z.shape
    P = N * H * W
    lb = L.lib()
    if pre is not None:
        part, R = pre
    else:
        R = lb.pmu_bn_bwd_tiles(P, C)
        part = _empty(R, 2 * C, device=dev)
        if da.dtype == BF16S and (z.dtype != F32 or C % 4 != 0):
            da = frame_to_f32([Src(da)], N, H, W)   # (the bf16-da reduce takes fp32 z, channel quads)
        name = ("pmu_bn_bwd_reduce_dxb" if da.dtype == BF16S else
                "pmu_bn_bwd_reduce_zb" if z.dtype == BF16S else "pmu_bn_bwd_reduce")
        L.call(name, da.data_ptr(), z.data_ptr(), st.coef.data_ptr(), st.mean.data_ptr(), st.invstd.data_ptr(), P, C,
               part.data_ptr(), s)
    G = lb.pmu_colsum_groups(R)
    acc = _empty(G, 2 * C, dtype=torch.float64, device=dev)
    L.call("pmu_colsum_f64", part.data_ptr(), R, 2 * C, acc.data_ptr(), G, s)
    dgamma = grads.new(bn.weight) if bn.weight is not None else None
    dbeta = grads.new(bn.bias) if bn.bias is not None else None
    dbias = grads.new(conv_bias) if conv_bias is not None else _empty(C, device=dev)
    bcoef = _empty(5 * C, device=dev)
    L.call("pmu_bn_bwd_finalize", acc.data_ptr(), G, C, float(P), L.ptr(bn.weight), st.coef.data_ptr(),
           st.mean.data_ptr(), st.invstd.data_ptr(), L.ptr(dgamma), L.ptr(dbeta), dbias.data_ptr(),
           bcoef.data_ptr(), s)
    return bcoef, dgamma, dbeta, dbias


# ----------------------------------------------------------------------------------------
# conv + BN layer
# ----------------------------------------------------------------------------------------
@dataclass
class ConvBNOut:
    z: torch.Tensor       # NHWC pre-BN conv output
    bn: BNState
    srcs: list = field(default_factory=list)   # the operand sources it consumed (for wgrad)
    planes: list | None = None                  # first-layer input planes
    bf16: bool = False                          # computed on the bf16-MFMA kernels
    xt: torch.Tensor | None = None              # bf16: the operand copy the forward kernel wrote (for wgrad)
    xt32: torch.Tensor | None = None            # fp32: the same, teed by pmu_conv3x3_fwd (RAW wgrad operand)
    bnr: tuple | None = None                    # (da, part, R): BN-backward partials formed by the consumer's dgrad

    def act(self, pool=L.POOL_NONE) -> Src:
        return Src(self.z, L.SRC_BNRELU, self.bn.coef, pool=pool, prod=self)


def first_layer_ok(cin: int, cout: int) -> bool:
    """Shapes pmu_conv_first_fwd/_wgrad take (include/pmunet_hip.h): Cin <= 4, Cout = 4q with 256 % q == 0."""
    return 1 <= cin <= 4 and cout % 4 == 0 and 4 <= cout <= 1024 and 256 % (cout // 4) == 0 and cout <= 256


def _check_channels(cin: int, layer) -> None:
    """The kernels take channel counts from the operand frame and index the weight by them, so an
    operand whose channel count differs from the layer's is refused here, as torch's conv would."""
    if cin != layer.in_channels:
        raise RuntimeError(f"{type(layer).__name__}: operand has {cin} channels, the layer expects "
                           f"{layer.in_channels} (weight {tuple(layer.weight.shape)})")


def conv_bn_forward(srcs, conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, N, H, W, training, dev,
                    planes=None, bf16=False, keep=False, zb=False) -> ConvBNOut:
    """relu(bn(conv(operand))) forward: z (pre-BN conv output, NHWC) + batch statistics.

    zb (bf16 mode, unet_forward with CFG.bf16_z): the LDS-DMA conv stores z in bf16, as torch.autocast
    keeps a conv's output, centred on the BN running mean (pmu_conv3x3_fwd_dma_zb: bf16(z - rm), so
    the rounding is relative to the channel's spread, not its mean); the layer's coefficients are
    then the centred ones (pmu_bn_center) and its consumers read z through bf16-aware frames,
    pmu_bn_bwd_reduce_zb, pmu_maxpool2_bwd_zb and the *_bnr_zb input gradient."""
    Cout = conv.out_channels
    _check_channels(len(planes) if planes is not None else sum(sr.C for sr in srcs), conv)
    s = L.stream()
    lb = L.lib()
    z = _empty(N, H, W, Cout, device=dev)
    xt = None
    zoff = None
    need_stats = training or not bn.track_running_stats
    if planes is not None and not first_layer_ok(len(planes), Cout):
        # channel counts outside the first-layer kernel: the generic 3x3 path on a raw NHWC frame
        srcs = [Src(torch.stack(planes, dim=-1).contiguous())]
        planes = None
    if planes is not None:
        R = lb.pmu_conv_first_tiles(N, H, W)
        part = _empty(R, 2 * Cout, device=dev) if need_stats else None
        arr = (ctypes.c_void_p * len(planes))(*[p.data_ptr() for p in planes])
        L.call("pmu_conv_first_fwd", arr, len(planes), N, H, W, conv.weight.data_ptr(), L.ptr(conv.bias), Cout,
               z.data_ptr(), L.ptr(part), s)
    elif bf16:
        Cp = _pad8(sum(sr.C for sr in srcs))
        use_dma = dma_ok(H, W, Cp, Cout, Cout)
        use_raw = use_dma or raw_ok(N, H, W, Cp)
        R = (lb.pmu_conv3x3_tiles_dma(N, H, W, Cout, Cp) if use_dma else
             lb.pmu_conv3x3_tiles_raw(N, H, W, Cout) if use_raw else lb.pmu_conv3x3_tiles(N, H, W))
        part = _empty(R, 2 * Cout, device=dev) if need_stats else None
        if use_dma:
            # both operands by LDS-DMA (maps >= 32 wide): the operand written once in bf16, as below
            xt = _materialised(srcs, BF16S)
            xt = xt if xt is not None else frame_to_bf16(srcs, N, H, W)
            wp = pack_weights_dma(conv.weight, dgrad=False)
            if zb and Cout % 8 == 0:   # (the bf16-z consumers take channel quads)
                z = _empty(N, H, W, Cout, dtype=BF16S, device=dev)
                # the running mean before this step's update (bn_forward below moves it)
                zoff = (bn.running_mean.detach().clone() if bn.track_running_stats and bn.running_mean is not None
                        else torch.zeros(Cout, device=dev))
                L.call("pmu_conv3x3_fwd_dma_zb", xt.data_ptr(), Cp, N, H, W, wp.data_ptr(), L.ptr(conv.bias), Cout,
                       z.data_ptr(), zoff.data_ptr(), L.ptr(part), s)
            else:
                L.call("pmu_conv3x3_fwd_dma", xt.data_ptr(), Cp, N, H, W, wp.data_ptr(), L.ptr(conv.bias), Cout,
                       z.data_ptr(), L.ptr(part), s)
            if not keep:
                xt = None
        elif use_raw:
            # the operand (BN+ReLU / max-pool / F.pad+cat applied) written once in bf16; the GEMM
            # streams it, and the weight gradient reuses it
            xt = _materialised(srcs, BF16S)
            xt = xt if xt is not None else frame_to_bf16(srcs, N, H, W)
            wp = pack_weights_raw(conv.weight, dgrad=False)
            L.call("pmu_conv3x3_fwd_raw", xt.data_ptr(), Cp, N, H, W, wp.data_ptr(), L.ptr(conv.bias), Cout,
                   z.data_ptr(), L.ptr(part), s)
            if not keep:
                xt = None
        else:
            wp = pack_weights_bf16(conv.weight, dgrad=False)
            xt = (torch.empty(N, H, W, Cp, dtype=torch.int16, device=dev)
                  if keep else None)   # the weight gradient's operand, teed by the fused kernel
            L.call("pmu_conv3x3_fwd_bf16", frame_of(_f32_srcs(srcs, N, H, W), N, H, W), wp.data_ptr(),
                   L.ptr(conv.bias), Cout, z.data_ptr(), L.ptr(part), L.ptr(xt), s)
    else:
        Cin = sum(sr.C for sr in srcs)
        # the weight gradient reads the operand the kernel staged (RAW) instead of re-deriving it
        xt32 = _empty(N, H, W, Cin, device=dev) if keep and tee32_ok(Cin, Cout) else None
        if use_wino() and wino4_ok(Cin, H, W, "fwd"):
            # F(4x4,3x3) on the materialised operand (images of >= 32 x 32)
            R = lb.pmu_conv3x3_tiles_wino4(N, H, W)
            part = _empty(R, 2 * Cout, device=dev) if need_stats else None
            wp = pack_weights_wino4(conv.weight, dgrad=False)
            xm = _materialised(srcs, F32)
            xm = xm if xm is not None else frame_to_f32(srcs, N, H, W)
            L.call("pmu_conv3x3_fwd_wino4", xm.data_ptr(), Cin, N, H, W, wp.data_ptr(), L.ptr(conv.bias),
                   Cout, z.data_ptr(), L.ptr(part), s)
            xt32 = xm if xt32 is not None else None
        elif use_wino():
            R = lb.pmu_conv3x3_tiles_wino(N, H, W)
            part = _empty(R, 2 * Cout, device=dev) if need_stats else None
            if wino_raw_ok(Cin) and wino2h_ok(Cin):
                # 1024-thread F(2x2) workgroups (four waves per SIMD) on the materialised operand
                xm = _materialised(srcs, F32)
                xm = xm if xm is not None else frame_to_f32(srcs, N, H, W)
                wp2 = pack_weights_wino2h(conv.weight, dgrad=False)
                L.call("pmu_conv3x3_fwd_wino2h", xm.data_ptr(), Cin, N, H, W, wp2.data_ptr(), L.ptr(conv.bias),
                       Cout, z.data_ptr(), L.ptr(part), s)
                xt32 = xm if xt32 is not None else None
            elif wino_raw_ok(Cin):
                # the operand materialised once (the weight gradient's operand anyway), then a
                # DMA-staged Winograd GEMM on it
                wp = pack_weights_wino(conv.weight, dgrad=False)
                xm = _materialised(srcs, F32)
                xm = xm if xm is not None else frame_to_f32(srcs, N, H, W)
                L.call("pmu_conv3x3_fwd_wino_raw", xm.data_ptr(), Cin, N, H, W, wp.data_ptr(), L.ptr(conv.bias),
                       Cout, z.data_ptr(), L.ptr(part), s)
                xt32 = xm if xt32 is not None else None
            else:
                wp = pack_weights_wino(conv.weight, dgrad=False)
                L.call("pmu_conv3x3_fwd_wino", frame_of(srcs, N, H, W), wp.data_ptr(), L.ptr(conv.bias), Cout,
                       z.data_ptr(), L.ptr(part), L.ptr(xt32), s)
        else:
            R = lb.pmu_conv3x3_tiles(N, H, W)
            part = _empty(R, 2 * Cout, device=dev) if need_stats else None
            wp = pack_weights(conv.weight, dgrad=False)
            L.call("pmu_conv3x3_fwd", frame_of(srcs, N, H, W), conv.weight.data_ptr(), wp.data_ptr(),
                   L.ptr(conv.bias), Cout, z.data_ptr(), L.ptr(part), L.ptr(xt32), s)
    st = bn_forward(part, R, Cout, N * H * W, bn, training, dev)
    if zoff is not None:   # consumers apply the coefficients to the centred stored z
        L.call("pmu_bn_center", st.coef.data_ptr(), L.ptr(st.mean), zoff.data_ptr(), Cout, st.coef.data_ptr(),
               L.ptr(st.mean), s)
    bfl = bf16 and planes is None
    return ConvBNOut(z=z, bn=st, srcs=list(srcs), planes=planes, bf16=bfl, xt=xt if bfl else None,
                     xt32=None if (bf16 or planes is not None) else xt32)


class PoolSumDa:
    """The gradient of a pooled layer's activation, da = dsk + routed dpool (MaxPool2d(2) backward,
    unet_parts.py:33, plus the skip path, unet_parts.py:66; both parts bf16 from *_dxb input gradients,
    or both fp32), left unstored: a stats-only max-pool pass (pmu_maxpool2_bwd_bnr_stats{_dxb,}) formed
    its BN-backward partial sums (prod.bnr) and dz() turns it into that layer's dz in one pass
    (pmu_maxpool2_bwd_bnbwd{_dxb,}: bf16 dz from bf16 parts, fp32 from fp32 ones) — the fp32 da is
    neither written nor re-read.  materialise() stores it (fp32) for the paths that read da itself."""

    def __init__(self, dpool: torch.Tensor, dsk: torch.Tensor, prod: ConvBNOut):
        self.dpool, self.dsk, self.prod = dpool, dsk, prod
        self.bf16_parts = dpool.dtype == BF16S
        self.shape = prod.z.shape
        self.dtype = F32
        self.device = prod.z.device

    def dz(self, bcoef: torch.Tensor, bf16: bool):
        """The layer's dz (bf16 bits or fp32), or None when the parts' storage does not match."""
        if bf16 != self.bf16_parts:
            return None
        N, H, W, C = self.shape
        dz = torch.empty(N, H, W, C, dtype=BF16S if bf16 else F32, device=self.device)
        L.call("pmu_maxpool2_bwd_bnbwd_dxb" if bf16 else "pmu_maxpool2_bwd_bnbwd", self.dpool.data_ptr(),
               self.dsk.data_ptr(), self.prod.z.data_ptr(), self.prod.bn.coef.data_ptr(), bcoef.data_ptr(), N, H, W, C,
               C, dz.data_ptr(), L.stream())
        return dz

    def dz_bf16(self, bcoef: torch.Tensor):
        return self.dz(bcoef, True)

    def materialise(self) -> torch.Tensor:
        N, H, W, C = self.shape
        p = self.prod
        part = _empty(L.lib().pmu_maxpool2_bwd_bnr_tiles(N, H, W, C), 2 * C, device=self.device)
        if self.bf16_parts:
            da = _empty(N, H, W, C, device=self.device)
            L.call("pmu_maxpool2_bwd_bnr_dxb", self.dpool.data_ptr(), self.dsk.data_ptr(), p.z.data_ptr(),
                   p.bn.coef.data_ptr(), p.bn.mean.data_ptr(), p.bn.invstd.data_ptr(), N, H, W, C, da.data_ptr(),
                   part.data_ptr(), L.stream())
        else:   # (the fp32 form accumulates in place: into a copy of the skip gradient)
            da = self.dsk.clone()
            L.call("pmu_maxpool2_bwd_bnr", self.dpool.data_ptr(), p.z.data_ptr(), p.bn.coef.data_ptr(),
                   p.bn.mean.data_ptr(), p.bn.invstd.data_ptr(), N, H, W, C, da.data_ptr(), 1, part.data_ptr(),
                   L.stream())
        return da


class HeadDa:
    """The last layer's activation gradient da = OutConv's input gradient (unet_parts.py:70-76 backward:
    sum over classes of dy_k w_k, through the sigmoid for one class) left unstored: the head backward
    (pmu_head1x1_bwd_bnr with da NULL) formed the layer's BN-backward partials and the head's weight
    gradient, and dz(bcoef, bf16) writes the layer's dz straight from dy (pmu_head1x1_bwd_dz) — the
    fp32 da is neither written nor re-read.  materialise() stores it for the paths that read da."""

    def __init__(self, dy: torch.Tensor, y: torch.Tensor, sigmoid: bool, w: torch.Tensor, K: int, prod: ConvBNOut):
        self.dy, self.y, self.sigmoid, self.w, self.K, self.prod = dy, y, sigmoid, w, K, prod
        self.shape = prod.z.shape
        self.dtype = F32
        self.device = prod.z.device

    def dz(self, bcoef: torch.Tensor, bf16: bool) -> torch.Tensor:
        N, H, W, C = self.shape
        out = torch.empty(N, H, W, C, dtype=BF16S if bf16 else F32, device=self.device)
        L.call("pmu_head1x1_bwd_dz", self.dy.data_ptr(), self.y.data_ptr(), int(self.sigmoid), self.w.data_ptr(),
               self.K, C, N, H, W, self.prod.z.data_ptr(), bcoef.data_ptr(), int(bf16), out.data_ptr(), L.stream())
        return out

    def dz_bf16(self, bcoef: torch.Tensor) -> torch.Tensor:
        return self.dz(bcoef, True)

    def materialise(self) -> torch.Tensor:
        N, H, W, C = self.shape
        da = _empty(N, H, W, C, device=self.device)
        dl = _empty(N, self.K, H, W, device=self.device)
        L.call("pmu_head1x1_bwd", self.dy.data_ptr(), self.y.data_ptr(), int(self.sigmoid), self.w.data_ptr(),
               self.K, C, N, H, W, dl.data_ptr(), da.data_ptr(), L.stream())
        return da


def pool_fuse_ok(C: int) -> bool:
    """Channel counts pmu_maxpool2_bwd_bnbwd_dxb takes: C % 4 == 0, C / 4 dividing 256 or a multiple of it."""
    q = C // 4
    return C % 4 == 0 and q > 0 and (256 % q == 0 if q < 256 else q % 256 == 0)


def _concrete(src: Src) -> Src:
    """src with a stored da (PoolSumDa / HeadDa materialised) for the kernels that read da itself."""
    if isinstance(src.x, (PoolSumDa, HeadDa)):
        return Src(src.x.materialise(), src.mode, src.coef, z=src.z, pool=src.pool, off=src.off, prod=src.prod)
    return src


def _bnr_producer(out: ConvBNOut, need_dx: bool, split):
    """The ConvBNOut whose BatchNorm+ReLU backward partial sums this conv's input gradient can form in
    its epilogue: the operand is that layer's unpooled activation alone and its batch statistics exist."""
    if not need_dx or split is not None or len(out.srcs) != 1:
        return None
    sr = out.srcs[0]
    p = sr.prod
    if sr.mode != L.SRC_BNRELU or sr.pool != L.POOL_NONE or p is None or p.bn.mean is None or sr.x is not p.z:
        return None
    return p


def tee32_ok(cin: int, cout: int) -> bool:
    """Channel counts for which the fp32 weight gradient runs on teed RAW operands (its 64x64 blocks)."""
    return cin % 64 == 0 and cout % 64 == 0


def conv_bn_backward(out: ConvBNOut, da: torch.Tensor, conv, bn, grads: dict, need_dx=True, split=None,
                     x1_bf16_only=False, dx_bf16=False):
    """Backward of relu(bn(conv(operand))) given da (NHWC; fp32, or bf16 bits from a *_dxb input
    gradient).  Writes conv/bn grads into ``grads``.

    Returns the operand gradient(s): one NHWC tensor, or (dx0, dx1) when ``split`` is given
    (channel split of a concatenated operand).  x1_bf16_only (bf16 convs): the caller needs dx1 only as
    the transposed conv's bf16 operand and its column sums (see _conv_backward_bf16).  dx_bf16 (bf16
    convs, CFG.dx_bf16): the caller's consumers take dx / dx0 stored as bf16 (BF16S) — the LDS-DMA input
    gradient then writes it so (autocast's dtype for a conv's input gradient)."""
    s = L.stream()
    z = out.z
    N, H, W, Cout = z.shape
    dev = z.device
    pre = None
    if out.bnr is not None and out.bnr[0] is da:
        pre = out.bnr[1:]
    out.bnr = None
    if pre is None and isinstance(da, (PoolSumDa, HeadDa)):
        da = da.materialise()
    bcoef, _, _, _ = bn_backward(da, z, out.bn, bn, grads, conv.bias, pre=pre)
    dz_src = Src(da, L.SRC_BNBWD, bcoef, z=z)
    dw = grads.new(conv.weight)
    lb = L.lib()
    prod = _bnr_producer(out, need_dx, split)
    if out.bf16:
        return _conv_backward_bf16(out, dz_src, conv, dw, need_dx, split, prod, x1_bf16_only, dx_bf16)
    # (an unstored head / pooled gradient gives dz itself, fp32: a RAW source of the same values)
    dzt = da.dz(bcoef, False) if isinstance(da, (HeadDa, PoolSumDa)) else None
    dz_src = Src(dzt) if dzt is not None else _concrete(dz_src)
    dzf = frame_of([dz_src], N, H, W)
    if out.xt32 is not None and need_dx:
        return _conv_backward_tee32(out, dz_src, conv, dw, split, prod)
    if out.planes is not None:
        Cin = len(out.planes)
        wsb = lb.pmu_conv_first_wgrad_ws(N, H, W, Cin, Cout)
        ws = _empty(max(1, (wsb + 3) // 4), device=dev)
        arr = (ctypes.c_void_p * Cin)(*[p.data_ptr() for p in out.planes])
        L.call("pmu_conv_first_wgrad", dzf, arr, Cin, Cout, dw.data_ptr(), ws.data_ptr(), wsb, s)
    else:
        Cin = sum(sr.C for sr in out.srcs)
        wsb = lb.pmu_conv3x3_wgrad_ws(N, H, W, Cin, Cout)
        ws = _empty(max(1, (wsb + 3) // 4), device=dev)
        L.call("pmu_conv3x3_wgrad", dzf, frame_of(out.srcs, N, H, W), Cout, dw.data_ptr(), ws.data_ptr(), wsb, s)
    if not need_dx or out.planes is not None:
        return None
    return _dgrad32(dz_src, conv, N, H, W, split, None, prod)


def _bnr_call(name, prod, R, lead, dx, s):
    """Launch a *_bnr input gradient (lead: its leading arguments up to Cin) and leave the producer's
    BN-backward partials on it for its own conv_bn_backward."""
    C = prod.z.shape[3]
    part = _empty(R, 2 * C, device=dx.device)
    L.call(name, *lead, dx.data_ptr(), prod.z.data_ptr(), prod.bn.coef.data_ptr(), prod.bn.mean.data_ptr(),
           prod.bn.invstd.data_ptr(), part.data_ptr(), s)
    prod.bnr = (dx, part, R)


def _dgrad32(dz_src, conv, N, H, W, split, tee, prod=None):
    """fp32 input gradient of a 3x3 conv (Winograd or direct); dx, or (dx0, dx1) split at ``split``.
    tee: receives dz (the BN+ReLU backward applied) for the weight gradient.  prod: the layer whose
    BN-backward partial sums the Winograd kernels form in their epilogue (see _bnr_producer)."""
    s = L.stream()
    dev = conv.weight.device
    Cin, Cout = conv.in_channels, conv.out_channels
    sp = Cin if split is None else split
    dx0 = _empty(N, H, W, sp, device=dev)
    dx1 = _empty(N, H, W, Cin - sp, device=dev) if split is not None else None
    if prod is not None and prod.z.dtype != F32:
        prod = None   # the fp32 kernels' BN-backward epilogue reads an fp32 z
    dz_src = _f32_srcs([dz_src], N, H, W)[0]
    dzf = frame_of([dz_src], N, H, W)
    lb = L.lib()
    # dz already stored in fp32 (an unstored head / pooled gradient's dz pass): read in place, no copy
    ready = _materialised([dz_src], F32)

    def dz_tensor():
        if ready is not None and (tee is None or tee is ready):
            return ready
        dzt = tee if tee is not None else _empty(N, H, W, Cout, device=dev)
        L.call("pmu_frame_to_f32", dzf, dzt.data_ptr(), s)
        return dzt
    if use_wino() and wino4_ok(Cout, H, W, "dgrad"):
        dzt = dz_tensor()
        wp = pack_weights_wino4(conv.weight, dgrad=True)
        if prod is not None:
            _bnr_call("pmu_conv3x3_dgrad_wino4_bnr", prod, lb.pmu_conv3x3_tiles_wino4(N, H, W),
                      (dzt.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin), dx0, s)
        else:
            L.call("pmu_conv3x3_dgrad_wino4", dzt.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, sp, dx0.data_ptr(),
                   L.ptr(dx1), s)
    elif use_wino() and wino_raw_ok(Cout) and wino2h_ok(Cout):
        dzt = dz_tensor()
        wp = pack_weights_wino2h(conv.weight, dgrad=True)
        if prod is not None:
            _bnr_call("pmu_conv3x3_dgrad_wino2h_bnr", prod, lb.pmu_conv3x3_tiles_wino2h(N, H, W),
                      (dzt.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin), dx0, s)
        else:
            L.call("pmu_conv3x3_dgrad_wino2h", dzt.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, sp, dx0.data_ptr(),
                   L.ptr(dx1), s)
    elif use_wino() and wino_raw_ok(Cout):
        dzt = dz_tensor()
        wp = pack_weights_wino(conv.weight, dgrad=True)
        L.call("pmu_conv3x3_dgrad_wino_raw", dzt.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, sp, dx0.data_ptr(),
               L.ptr(dx1), s)
    else:
        tee = None if (ready is not None and tee is ready) else tee   # (the tee would be the source itself)
        if use_wino():
            wp = pack_weights_wino(conv.weight, dgrad=True)
            L.call("pmu_conv3x3_dgrad_wino", dzf, wp.data_ptr(), Cin, sp, dx0.data_ptr(), L.ptr(dx1), L.ptr(tee), s)
        else:
            wp = pack_weights(conv.weight, dgrad=True)
            L.call("pmu_conv3x3_dgrad", dzf, conv.weight.data_ptr(), wp.data_ptr(), Cin, sp, dx0.data_ptr(),
                   L.ptr(dx1), L.ptr(tee), s)
    return dx0 if split is None else (dx0, dx1)


def _conv_backward_tee32(out: ConvBNOut, dz_src, conv, dw, split, prod=None):
    """fp32 backward with materialised operands: the input-gradient kernel tees dz (BN+ReLU backward
    applied) as it stages it, and the weight gradient multiplies that with the operand the forward
    teed — both RAW frames, so its staging is a plain copy."""
    s = L.stream()
    lb = L.lib()
    N, H, W, Cout = out.z.shape
    dev = out.z.device
    Cin = conv.in_channels
    # (a dz already stored in fp32 is the tee itself)
    dzt = _materialised([dz_src], F32)
    dzt = dzt if dzt is not None else _empty(N, H, W, Cout, device=dev)
    res = _dgrad32(dz_src, conv, N, H, W, split, dzt, prod)
    wsb4 = (lb.pmu_conv3x3_wgrad_ws_wino4(N, H, W, Cin, Cout)
            if (use_wino() and CFG.wgrad4 and L.experiments_build()) else 0)
    wsb = 0 if wsb4 else (lb.pmu_conv3x3_wgrad_ws_wino(N, H, W, Cin, Cout) if use_wino() else 0)
    if wsb4:
        ws = _empty((wsb4 + 3) // 4, device=dev)
        L.call("pmu_conv3x3_wgrad_wino4", dzt.data_ptr(), out.xt32.data_ptr(), N, H, W, Cout, Cin, dw.data_ptr(),
               ws.data_ptr(), wsb4, s)
    elif wsb:
        ws = _empty((wsb + 3) // 4, device=dev)
        L.call("pmu_conv3x3_wgrad_wino", dzt.data_ptr(), out.xt32.data_ptr(), N, H, W, Cout, Cin, dw.data_ptr(),
               ws.data_ptr(), wsb, s)
    else:
        wsb = lb.pmu_conv3x3_wgrad_ws(N, H, W, Cin, Cout)
        ws = _empty(max(1, (wsb + 3) // 4), device=dev)
        L.call("pmu_conv3x3_wgrad", frame_of([Src(dzt)], N, H, W), frame_of([Src(out.xt32)], N, H, W), Cout,
               dw.data_ptr(), ws.data_ptr(), wsb, s)
    out.xt32 = None
    return res


def _pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def frame_to_bf16(srcs, N, H, W) -> torch.Tensor:
    """The bf16 operand of a frame, NHWC with channels padded to a multiple of 8 (pmu_frame_to_bf16)."""
    C = sum(sr.C for sr in srcs)
    out = torch.empty(N, H, W, _pad8(C), dtype=torch.int16, device=srcs[0].x.device)
    L.call("pmu_frame_to_bf16", frame_of(srcs, N, H, W), _pad8(C), out.data_ptr(), L.stream())
    return out


def raw_ok(N, H, W, Cp) -> bool:
    """Shapes the materialised-operand bf16 conv takes (pmu_conv3x3_fwd_raw / _dgrad_raw)."""
    return N * H * W * Cp < 2 ** 31


def _conv_backward_bf16(out: ConvBNOut, dz_src: Src, conv, dw, need_dx, split, prod=None, x1_bf16_only=False,
                        dx_bf16=False):
    """bf16-MFMA backward of one conv layer (torch.autocast(bfloat16) arithmetic).  dz after the
    BN+ReLU backward is written once in bf16 (dzt); the input gradient streams it (or, for a concat
    split that is not a multiple of 32, stages dz's frame in the fused kernel) and the weight
    gradient multiplies it with the forward's bf16 operand (out.xt)."""
    s = L.stream()
    N, H, W, Cout = out.z.shape
    dev = out.z.device
    Cin = conv.in_channels
    dzt = dz_src.x.dz_bf16(dz_src.coef) if isinstance(dz_src.x, (PoolSumDa, HeadDa)) else None
    if dzt is None:
        dz_src = _concrete(dz_src)
        dzt = frame_to_bf16([dz_src], N, H, W)
    res = None
    if need_dx:
        sp = Cin if split is None else split
        use_dma = dma_ok(H, W, dzt.shape[3], Cin, sp)
        # bf16 dx0 (the *_dxb entries; every other output formed from the rounded values)
        xb = dx_bf16 and CFG.dx_bf16 and dxb_ok(H, W, Cout, Cin, sp)
        dx0 = _empty(N, H, W, sp, dtype=BF16S if xb else F32, device=dev)
        sfx = "_dxb" if xb else ""
        x1only = x1_bf16_only and sp < Cin and (Cin - sp) % 8 == 0 and use_dma
        dx1 = _empty(N, H, W, Cin - sp, device=dev) if sp < Cin and not x1only else None
        if x1only:
            # dx1 only in bf16 (the transposed conv's operand) with per-tile column sums (its bias gradient):
            # the fp32 dx1 is neither written nor re-read
            wp = pack_weights_dma(conv.weight, dgrad=True)
            R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3])
            part = _empty(R, 2 * Cin, device=dev)
            dx1 = torch.empty(N, H, W, Cin - sp, dtype=BF16S, device=dev)
            L.call("pmu_conv3x3_dgrad_dma_x1b_sum" + sfx, dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin,
                   sp, dx0.data_ptr(), dx1.data_ptr(), part.data_ptr(), s)
            dx1._pmu_dbpart = (part, R, sp)
        elif use_dma:
            wp = pack_weights_dma(conv.weight, dgrad=True)
            if prod is not None:
                if prod.z.dtype == BF16S:   # (experiments build: bf16 z; its dx stays fp32)
                    dx0 = _empty(N, H, W, sp, device=dev) if xb else dx0
                    name = "pmu_conv3x3_dgrad_dma_bnr_zb"
                else:
                    name = "pmu_conv3x3_dgrad_dma_bnr" + sfx
                _bnr_call(name, prod, L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3]),
                          (dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin), dx0, s)
            elif dx1 is not None and (Cin - sp) % 8 == 0:
                # the up-sampled part's gradient also in bf16: the transposed conv's operand, kept on the
                # fp32 tensor (unet_backward uses it instead of a pmu_frame_to_bf16 pass over dx1)
                dx1b = torch.empty(N, H, W, Cin - sp, dtype=BF16S, device=dev)
                L.call("pmu_conv3x3_dgrad_dma_x1b" + sfx, dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin,
                       sp, dx0.data_ptr(), dx1.data_ptr(), dx1b.data_ptr(), s)
                dx1._pmu_bf16 = dx1b
            else:
                L.call("pmu_conv3x3_dgrad_dma" + sfx, dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, sp,
                       dx0.data_ptr(), L.ptr(dx1), s)
        elif raw_ok(N, H, W, dzt.shape[3]) and (sp == Cin or sp % 32 == 0):
            wp = pack_weights_raw(conv.weight, dgrad=True)
            L.call("pmu_conv3x3_dgrad_raw", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, sp,
                   dx0.data_ptr(), L.ptr(dx1), s)
        else:
            wp = pack_weights_bf16(conv.weight, dgrad=True)
            dz_src = _concrete(dz_src)
            L.call("pmu_conv3x3_dgrad_bf16", frame_of(_f32_srcs([dz_src], N, H, W), N, H, W), wp.data_ptr(), Cin,
                   sp, dx0.data_ptr(), L.ptr(dx1), None, s)
        res = dx0 if split is None else (dx0, dx1)
    xt = out.xt if out.xt is not None else frame_to_bf16(out.srcs, N, H, W)
    out.xt = None
    lb = L.lib()
    sfx = "_dma" if CFG.wgrad_dma and lb.pmu_conv3x3_wgrad_dma_ok(N, H, W, Cin, Cout) else ""
    wsb = getattr(lb, "pmu_conv3x3_wgrad_ws_bf16" + sfx)(N, H, W, Cin, Cout)
    ws = _empty(max(1, (wsb + 3) // 4), device=dev)
    L.call("pmu_conv3x3_wgrad_bf16" + sfx, dzt.data_ptr(), xt.data_ptr(), N, H, W, Cout, Cin, dw.data_ptr(),
           ws.data_ptr(), wsb, s)
    return res


def dxb_ok(H, W, Cout, Cin, split) -> bool:
    """The conv's input gradient runs on the LDS-DMA kernel and may store dx in bf16 (the *_dxb entries):
    maps >= 32 wide, pad8(Cout) % 16 == 0, a concat split on a 32-channel boundary, Cin and the split
    multiples of 8.  oracle/unet_ref.py's _dma_dxb models the same rule (tests/test_cpu_host.py)."""
    return dma_ok(H, W, _pad8(Cout), Cin, split) and Cin % 8 == 0 and split % 8 == 0


def dma_ok(H, W, Cp, NOUT, split) -> bool:
    """Shapes of the LDS-DMA bf16 conv (pmu_conv3x3_{fwd,dgrad}_dma): maps >= 32 wide, Cp % 16 == 0,
    a concat split on a 32-channel boundary."""
    return bool(L.lib().pmu_conv3x3_dma_ok(H, W, Cp, NOUT, split))


def _pack_weights_dma_now(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """Weights rounded to bf16 in the LDS-DMA conv's swizzled unit order (pmu_conv3x3_pack_dma)."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size_dma(Cout, Cin, int(dgrad)) // 2
    wp = torch.empty(n, dtype=torch.int16, device=w.device)
    L.call("pmu_conv3x3_pack_dma", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def pack_weights_raw(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """Weights rounded to bf16 in the materialised-operand conv's B tiles (pmu_conv3x3_pack_raw)."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size_raw(Cout, Cin, int(dgrad)) // 2
    wp = torch.empty(n, dtype=torch.int16, device=w.device)
    L.call("pmu_conv3x3_pack_raw", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def pack_weights_bf16(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """Weights rounded to bf16 and laid out as the bf16 conv kernel's B tiles (pmu_conv3x3_pack_bf16)."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size_bf16(Cout, Cin, int(dgrad)) // 2
    wp = torch.empty(n, dtype=torch.int16, device=w.device)
    L.call("pmu_conv3x3_pack_bf16", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def pack_weights_wino(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """Winograd-transformed weights U = G g G^T in the fp32 Winograd kernel's blocks (pmu_conv3x3_pack_wino)."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size_wino(Cout, Cin, int(dgrad)) // 4
    wp = _empty(n, device=w.device)
    L.call("pmu_conv3x3_pack_wino", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def _pack_weights_wino4_now(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """F(4x4,3x3) weights U = G g G^T in the F(4x4) kernel's blocks (pmu_conv3x3_pack_wino4)."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size_wino4(Cout, Cin, int(dgrad)) // 4
    wp = _empty(n, device=w.device)
    L.call("pmu_conv3x3_pack_wino4", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


@dataclass
class EngineConfig:
    """Implementation choices of the fp32 3x3 convs, read ONCE from the environment at import (never
    on the per-call hot path).  Tests switch them by assigning ``CFG``'s fields.

    fp32_conv: "wino" (default: Winograd on materialised operands), "wino_fused" (the fused-staging
        Winograd kernels everywhere) or "direct" (direct-sum MFMA kernels) — PMU_FP32_CONV;
    wino2h: the 1024-thread F(2x2) kernels (default) or the 512-thread ones — PMU_WINO2H=0;
    wino4: where F(4x4,3x3) runs — "dgrad" (default: the input gradient of maps >= 32x32) or "0"
        (nowhere) — PMU_WINO4.  "1" (the forward too) breaks the model-level 1e-3 contract (see
        wino4_ok) and is honoured only by an experiments build of the library (make EXPERIMENTS=1);
    bf16_z: bf16 mode (unet_forward) stores the LDS-DMA convs' pre-BN output z in bf16, centred on the
        BN running mean — the dtype torch.autocast gives a conv's output.  Off by default: it breaks
        the c5 Dice contract (eval Dice gap 6.8e-3 centred / 5.4e-3 uncentred vs 2.2e-4 with fp32 z,
        tests/test_bf16_gpu.py::test_c5_bf16_dice_gap_vs_fp32_oracle), so PMU_BF16_Z=1
        is honoured only by an experiments build of the library, as PMU_WINO4=1;
    wgrad4: the fp32 weight gradient by Winograd F(4x4,3x3) where its shapes allow (PMU_WGRAD4=1; off by
        default: measured equal to F(2x2) over the c2 shapes, 10.29 vs 10.29 ms — LDS-read bound);
    dx_bf16: bf16 mode keeps the activation gradients the LDS-DMA input gradients produce inside the
        UNet backward in bf16 (the *_dxb entries) — the dtype torch.autocast's conv backward returns
        them in — and their consumers read them so (PMU_DX_BF16=0: fp32, the round-4 path);
    wgrad_dma: the bf16 weight gradient on the LDS-DMA strip kernel (pmu_conv3x3_wgrad_bf16_dma) where
        its shapes allow, else the register-staged one (PMU_WGRAD_DMA=0: always the latter);
    pool_fuse: a pooled layer's da (skip + routed pooled gradient, both bf16) is not stored: a
        stats-only pass forms its BN-backward partials and its bf16 dz is made from the two parts
        directly (PoolSumDa; PMU_POOL_FUSE=0: stored in fp32 and streamed, the round-5 path);
    head_fuse: the head's input gradient (the last layer's da) is not stored: the head backward forms
        the last layer's BN-backward partials and the head's weight gradient, and that layer's dz (bf16 or
        fp32) is made from dy directly (HeadDa; PMU_HEAD_FUSE=0: da stored, then streamed);
    prob_streams: the Probabilistic U-Net's forward runs its UNet, prior and posterior on three HIP
        streams (functions.run_concurrent; their backwards follow autograd's stream of the forward), so
        the parts' tile-starved deep layers and small launches overlap (PMU_PROB_STREAMS=0: one stream)."""
    fp32_conv: str = "wino"
    wino2h: bool = True
    wino4: str = "dgrad"
    bf16_z: bool = False
    wgrad4: bool = False
    dx_bf16: bool = True
    wgrad_dma: bool = True
    pool_fuse: bool = True
    head_fuse: bool = True
    prob_streams: bool = True

    @classmethod
    def from_env(cls):
        return cls(fp32_conv=os.environ.get("PMU_FP32_CONV", "wino"), wino2h=os.environ.get("PMU_WINO2H", "1") != "0",
                   wino4=os.environ.get("PMU_WINO4", "dgrad"), bf16_z=os.environ.get("PMU_BF16_Z", "0") == "1",
                   wgrad4=os.environ.get("PMU_WGRAD4", "0") == "1", dx_bf16=os.environ.get("PMU_DX_BF16", "1") != "0",
                   wgrad_dma=os.environ.get("PMU_WGRAD_DMA", "1") != "0",
                   pool_fuse=os.environ.get("PMU_POOL_FUSE", "1") != "0",
                   head_fuse=os.environ.get("PMU_HEAD_FUSE", "1") != "0",
                   prob_streams=os.environ.get("PMU_PROB_STREAMS", "1") != "0")


CFG = EngineConfig.from_env()


def wino4_ok(C: int, H: int, W: int, kind: str) -> bool:
    """Winograd F(4x4,3x3) on a materialised operand (pmu_conv3x3_*_wino4): reduction channels C % 8 == 0
    and images of at least 32 x 32 (its blocks are 32 x 32 output pixels; smaller maps keep F(2x2)).

    Default: the input gradient only.  F(4x4)'s fp32 rounding (~1e-6 relative rms, 5-10x the direct
    sum's; tools/wino_err.py) is harmless in the input gradient (c5 12-step Dice gap 2.7e-4 vs 2.2e-4
    with F(2x2)), but in the forward it enters the BatchNorm statistics: BN's backward amplifies it by
    |z|/sigma per element (UNet at batch 2 of 64x48: weight gradients 2.6e-3 of their max, F(2x2)
    7.9e-4) and the running statistics carry it into eval mode (c5 12-step eval Dice gap 1.13e-3 > the
    1e-3 contract).  The forward on F(4x4) (CFG.wino4 == "1") is therefore an experiments-build A/B
    only (kernel parity in tests/test_wino4_gpu.py)."""
    mode = CFG.wino4
    if mode == "1" and not L.experiments_build():
        mode = "dgrad"
    return C % 8 == 0 and H >= 32 and W >= 32 and (mode == "1" or mode == kind) and fp32_mode() == "wino"


def _pack_weights_wino2h_now(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """F(2x2,3x3) weights in the 1024-thread kernel's 64-channel blocks (pmu_conv3x3_pack_wino2h)."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size_wino2h(Cout, Cin, int(dgrad)) // 4
    wp = _empty(n, device=w.device)
    L.call("pmu_conv3x3_pack_wino2h", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def wino2h_ok(C: int) -> bool:
    """The 1024-thread F(2x2) kernels (pmu_conv3x3_{fwd,dgrad}_wino2h; four waves per SIMD where the
    512-thread raw kernel runs two): C % 8 == 0.  kbench on the c2 shapes: forward 11.57 -> 10.98 ms
    (256x256 layers 1.04 -> 0.90 ms).  CFG.wino2h False: the 512-thread raw kernels."""
    return C % 8 == 0 and (CFG.wino2h or not L.experiments_build())


def fp32_mode() -> str:
    """CFG.fp32_conv as honoured by the loaded library: "direct" (the direct-sum kernels) exists only in an
    experiments build; the shipped library runs the default Winograd path instead."""
    if CFG.fp32_conv == "direct" and not L.experiments_build():
        return "wino"
    return CFG.fp32_conv


def use_wino() -> bool:
    """fp32 3x3 convs (fwd and input gradient) by Winograd (fp32_mode() "direct": the direct sum)."""
    return fp32_mode() != "direct"


def wino_raw_ok(C: int) -> bool:
    """Winograd on a materialised operand (pmu_conv3x3_*_wino_raw): C % 16 == 0 (CFG.fp32_conv
    "wino_fused" keeps the fused-staging Winograd kernels)."""
    return C % 16 == 0 and fp32_mode() == "wino"


def frame_to_f32(srcs, N, H, W) -> torch.Tensor:
    """The fp32 operand of a frame, materialised NHWC (pmu_frame_to_f32)."""
    C = sum(sr.C for sr in srcs)
    out = _empty(N, H, W, C, device=srcs[0].x.device)
    L.call("pmu_frame_to_f32", frame_of(srcs, N, H, W), out.data_ptr(), L.stream())
    return out


def pack_weights(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """Weights re-laid out as the conv kernel's per-block B tiles (pmu_conv3x3_pack); one launch,
    ~2x the weight bytes of traffic, so staging inside the conv is a straight copy."""
    Cout, Cin = w.shape[0], w.shape[1]
    n = L.lib().pmu_conv3x3_packed_size(Cout, Cin, int(dgrad)) // 4
    wp = _empty(n, device=w.device)
    L.call("pmu_conv3x3_pack", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def _pack_convT_weights_dma_now(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """ConvT weights rounded to bf16 in the LDS-DMA GEMMs' swizzled unit order (pmu_convT2x2_pack_dma)."""
    Cin, Cout = w.shape[0], w.shape[1]
    wp = torch.empty(L.lib().pmu_convT2x2_packed_size_dma(Cin, Cout) // 2, dtype=torch.int16, device=w.device)
    L.call("pmu_convT2x2_pack_dma", w.data_ptr(), Cin, Cout, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def pack_convT_weights_bf16(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """ConvT weights rounded to bf16 in pmu_convT2x2_pack's layouts (pmu_convT2x2_pack_bf16)."""
    Cin, Cout = w.shape[0], w.shape[1]
    wp = torch.empty(4 * Cin * Cout, dtype=torch.int16, device=w.device)
    L.call("pmu_convT2x2_pack_bf16", w.data_ptr(), Cin, Cout, int(dgrad), wp.data_ptr(), L.stream())
    return wp


def _pack_convT_weights_now(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """ConvT weights [Cin][Cout][2][2] re-laid out k-contiguous for the pipelined GEMMs (pmu_convT2x2_pack)."""
    Cin, Cout = w.shape[0], w.shape[1]
    wp = _empty(L.lib().pmu_convT2x2_packed_size(Cin, Cout) // 4, device=w.device)
    L.call("pmu_convT2x2_pack", w.data_ptr(), Cin, Cout, int(dgrad), wp.data_ptr(), L.stream())
    return wp


# ----------------------------------------------------------------------------------------
# U-Net
# ----------------------------------------------------------------------------------------
def _dc_layers(dc):
    """(conv1, bn1, conv2, bn2) of a DoubleConv (double_conv = [conv, bn, relu, conv, bn, relu])."""
    s = dc.double_conv
    return s[0], s[1], s[3], s[4]


@dataclass
class UpState:
    u: torch.Tensor | None   # convT output, NHWC [N][2h][2w][Cup] (None: written into the concat operand)
    off: tuple               # (pad_top, pad_left) inside the skip frame
    prev: ConvBNOut          # convT input producer
    c1: ConvBNOut
    c2: ConvBNOut
    bf16: bool = False       # convT input gradient on bf16 MFMA where its shapes allow
    xt: torch.Tensor | None = None   # bf16: the convT operand the forward materialised (weight gradient)
    cskip: int = 0                   # channels of the skip half of the concat operand (backward split)


class UNetState:
    """Everything the backward needs from one forward."""

    def __init__(self):
        self.xcat = {}          # level -> Up-block concat operand whose skip half the encoder wrote
        self.x = None
        self.planes = None
        self.enc: list = []     # per level: (c1, c2) ConvBNOut
        self.ups: list = []     # per up block: UpState
        self.y = None           # head output (NCHW)
        self.feat_src = None    # last DoubleConv output producer


def _convT_ld_ok(N, h, w, cin, cout, ptr) -> bool:
    """The decoder's in-place fp32 transposed conv (pmu_convT2x2_fwd_ld) takes an N x h x w x cin
    BN+ReLU input producing cout channels — the test unet_forward's decoder applies to its actual
    input frame, asked ahead of time by the encoder (ptr: any device pointer; not dereferenced)."""
    f = L.PmuFrame()
    f.nsrc, f.N, f.H, f.W = 1, N, h, w
    c = f.src[0]
    c.x = c.coef = ptr
    c.mode, c.pool, c.dtype = L.SRC_BNRELU, L.POOL_NONE, 0
    c.C, c.H, c.W = cin, h, w
    return bool(L.lib().pmu_convT2x2_fwd_ld_ok(ctypes.byref(f), cout))


def _pool_skip(up, prev: ConvBNOut, srcs, N, h, w, bf16):
    """(pooled operand, concat operand) from one pass over prev's activation
    (pmu_frame_to_*_pool_skip), when the Up block that takes prev as its skip will build its concat
    operand in place (see unet_forward's decoder: no F.pad, 8-channel halves, the conv staging a
    materialised operand); else None.  The concat tensor's other half is the transposed conv's."""
    if prev.z.dtype != F32 or 2 * h != prev.z.shape[1] or 2 * w != prev.z.shape[2]:
        return None
    Cskip, Cup = prev.z.shape[3], up.up.out_channels
    Ccat, Cout1 = Cskip + Cup, _dc_layers(up.conv)[0].out_channels
    hs, ws_ = 2 * h, 2 * w
    if Cskip % 8 or Cup % 8:
        return None
    lb = L.lib()
    if bf16:
        if not (lb.pmu_convT2x2_dma_ok(up.up.in_channels, Cup, 0) and dma_ok(hs, ws_, Ccat, Cout1, Cout1)
                and (dma_ok(h, w, Cskip, Cout1, Cout1) or raw_ok(N, h, w, Cskip))):
            return None
    elif not (use_wino() and (wino4_ok(Ccat, hs, ws_, "fwd") or wino_raw_ok(Ccat))
              and _convT_ld_ok(N, h, w, up.up.in_channels, Cup, prev.z.data_ptr())):
        return None   # (the decoder then builds its concat operand from u: the skip half would go unread)
    f = frame_of(srcs, N, h, w)
    if not lb.pmu_frame_pool_skip_ok(f):
        return None
    dev = prev.z.device
    dt = BF16S if bf16 else F32
    pooled = torch.empty(N, h, w, Cskip, dtype=dt, device=dev)
    xcat = torch.empty(N, hs, ws_, Ccat, dtype=dt, device=dev)
    L.call("pmu_frame_to_bf16_pool_skip" if bf16 else "pmu_frame_to_f32_pool_skip", f, pooled.data_ptr(),
           xcat.data_ptr(), Ccat, L.stream())
    return pooled, xcat


def unet_forward(net, x: torch.Tensor, training: bool, bf16: bool = False, keep: bool = False):
    """Forward of model.UNet on the HIP path.  Returns (output, state).

    Output: NCHW logits / sigmoid(logits) when net.apply_last_layer, else the last
    DoubleConv activation as an NCHW-shaped channels-last tensor (unet_model.py:48-54).
    bf16: the 3x3 convs (except the Cin <= 4 first layer) and the ConvTranspose2d forward / input
    gradient (where their shapes allow) run on the bf16-MFMA kernels (autocast arithmetic; see
    include/pmunet_hip.h), the 3x3 weight gradients too.  keep: a backward follows (bf16 convs keep
    their operand copies for the weight gradient)."""
    assert x.is_cuda and x.dtype == F32 and x.dim() == 4
    dev = x.device
    N, Cin, H, W = x.shape
    st = UNetState()
    st.x = x
    # first layer reads NCHW planes directly (C == 1 is also NHWC)
    xc = x.contiguous()
    if Cin <= 4:
        st.planes = [xc[:, c] for c in range(Cin)]
        planes = [p if p.is_contiguous() else p.contiguous() for p in st.planes]
        st.planes = planes
        first_srcs = []
    else:
        planes = None
        first_srcs = [Src(xc.permute(0, 2, 3, 1).contiguous())]
    # ---- encoder
    c1w, b1, c2w, b2 = _dc_layers(net.inc)
    zb = bf16 and CFG.bf16_z and L.experiments_build()
    o1 = conv_bn_forward(first_srcs, c1w, b1, N, H, W, training, dev, planes=planes, bf16=bf16, keep=keep, zb=zb)
    o2 = conv_bn_forward([o1.act()], c2w, b2, N, H, W, training, dev, bf16=bf16, keep=keep, zb=zb)
    st.enc.append((o1, o2))
    h, w = H, W
    nlev = len(net.down_blocks) + 1
    for down in net.down_blocks:
        dc = down.maxpool_conv[1]
        c1w, b1, c2w, b2 = _dc_layers(dc)
        prev = st.enc[-1][1]
        h, w = h // 2, w // 2
        srcs = [prev.act(L.POOL_MAX2)]
        pre = _pool_skip(net.up_blocks[nlev - 2 - (len(st.enc) - 1)], prev, srcs, N, h, w, bf16)
        if pre is not None:
            # the pooled operand and the Up block's concat operand (skip half) in one pass over prev
            srcs = [Src(pre[0])]
            st.xcat[len(st.enc) - 1] = pre[1]
        elif bf16 and not raw_ok(N, h, w, _pad8(prev.z.shape[3])):
            # fused bf16 fallback: the max-pooled activation materialised once, read raw by every
            # column block (the pipelined fused kernel has no pooled staging)
            pooled = _empty(N, h, w, prev.z.shape[3], device=dev)
            L.call("pmu_frame_to_f32", frame_of(srcs, N, h, w), pooled.data_ptr(), L.stream())
            srcs = [Src(pooled)]
        o1 = conv_bn_forward(srcs, c1w, b1, N, h, w, training, dev, bf16=bf16, keep=keep, zb=zb)
        o2 = conv_bn_forward([o1.act()], c2w, b2, N, h, w, training, dev, bf16=bf16, keep=keep, zb=zb)
        st.enc.append((o1, o2))
    # ---- decoder
    cur = st.enc[-1][1]
    nlev = len(st.enc)
    for j, up in enumerate(net.up_blocks):
        skip = st.enc[nlev - 2 - j][1]
        xpre = st.xcat.pop(nlev - 2 - j, None)
        hs, ws_ = skip.z.shape[1], skip.z.shape[2]
        hi, wi = cur.z.shape[1], cur.z.shape[2]
        convT = up.up
        Cup = convT.out_channels
        fin = frame_of([cur.act()], N, hi, wi)
        Cin_t = cur.z.shape[3]
        _check_channels(Cin_t, convT)
        xtT = None
        dY, dX = hs - 2 * hi, ws_ - 2 * wi
        assert dY >= 0 and dX >= 0, "decoder feature map larger than skip (unsupported by reference too)"
        off = (dY // 2, dX // 2)
        c1w, b1, c2w, b2 = _dc_layers(up.conv)
        Cskip = skip.z.shape[3]
        Ccat = Cskip + Cup
        lb = L.lib()
        # The concat operand built in place: the transposed conv writes its half (channels Cskip..) of
        # the materialised operand directly and only the skip half is copied (no u tensor, one pass over
        # it less) — when the halves need no F.pad and the conv will stage a materialised operand.
        direct = dY == 0 and dX == 0 and Cskip % 8 == 0 and Cup % 8 == 0 and skip.z.dtype == F32
        if bf16:
            direct = (direct and bool(lb.pmu_convT2x2_dma_ok(Cin_t, Cup, 0)) and
                      dma_ok(hs, ws_, Ccat, c1w.out_channels, c1w.out_channels))
        else:
            direct = (direct and use_wino() and (wino4_ok(Ccat, hs, ws_, "fwd") or wino_raw_ok(Ccat)) and
                      bool(lb.pmu_convT2x2_fwd_ld_ok(fin, Cup)))
        # (xpre: the encoder already wrote the skip half, with the next level's pooled operand)
        ready = xpre is not None and xpre.shape == (N, hs, ws_, Ccat) and xpre.dtype == (BF16S if bf16 else F32)
        if direct and bf16:
            xcat = xpre if ready else torch.empty(N, hs, ws_, Ccat, dtype=BF16S, device=dev)
            xtT = frame_to_bf16([cur.act()], N, hi, wi)
            wpt = pack_convT_weights_dma(convT.weight, dgrad=False)
            L.call("pmu_convT2x2_fwd_dma_ldb", xtT.data_ptr(), xtT.shape[3], N, hi, wi, wpt.data_ptr(),
                   L.ptr(convT.bias), Cin_t, Cup, xcat.data_ptr() + 2 * Cskip, Ccat, L.stream())
            if not ready:
                L.call("pmu_frame_to_bf16_ld", frame_of([skip.act()], N, hs, ws_), Cskip, xcat.data_ptr(), Ccat,
                       L.stream())
            if not keep:
                xtT = None
            u, srcs = None, [Src(xcat)]
        elif direct:
            xcat = xpre if ready else _empty(N, hs, ws_, Ccat, device=dev)
            wpt = pack_convT_weights(convT.weight, dgrad=False)
            L.call("pmu_convT2x2_fwd_ld", fin, convT.weight.data_ptr(), wpt.data_ptr(), L.ptr(convT.bias), Cup,
                   xcat.data_ptr() + 4 * Cskip, Ccat, L.stream())
            if not ready:
                L.call("pmu_frame_to_f32_ld", frame_of([skip.act()], N, hs, ws_), xcat.data_ptr(), Ccat, L.stream())
            u, srcs = None, [Src(xcat)]
        else:
            u = _empty(N, 2 * hi, 2 * wi, Cup, device=dev)
            if bf16 and lb.pmu_convT2x2_dma_ok(Cin_t, Cup, 0):
                # the BN+ReLU operand written once in bf16 (the weight gradient's operand too), both GEMM
                # operands by LDS-DMA
                xtT = frame_to_bf16([cur.act()], N, hi, wi)
                wpt = pack_convT_weights_dma(convT.weight, dgrad=False)
                L.call("pmu_convT2x2_fwd_dma", xtT.data_ptr(), xtT.shape[3], N, hi, wi, wpt.data_ptr(),
                       L.ptr(convT.bias), Cin_t, Cup, u.data_ptr(), L.stream())
                if not keep:
                    xtT = None
            elif bf16 and L.experiments_build() and lb.pmu_convT2x2_bf16_ok(fin, Cup):   # (same shapes as the DMA one)
                wpt = pack_convT_weights_bf16(convT.weight, dgrad=False)
                L.call("pmu_convT2x2_fwd_bf16", fin, wpt.data_ptr(), L.ptr(convT.bias), Cup, u.data_ptr(), L.stream())
            else:
                wpt = pack_convT_weights(convT.weight, dgrad=False)
                L.call("pmu_convT2x2_fwd", frame_of(_f32_srcs([cur.act()], N, hi, wi), N, hi, wi),
                       convT.weight.data_ptr(), wpt.data_ptr(), L.ptr(convT.bias), Cup, u.data_ptr(), L.stream())
            srcs = [skip.act(), Src(u, L.SRC_RAW, off=off)]
        o1 = conv_bn_forward(srcs, c1w, b1, N, hs, ws_, training, dev, bf16=bf16, keep=keep, zb=zb)
        o2 = conv_bn_forward([o1.act()], c2w, b2, N, hs, ws_, training, dev, bf16=bf16, keep=keep, zb=zb)
        st.ups.append(UpState(u=u, off=off, prev=cur, c1=o1, c2=o2, bf16=bf16, xt=xtT, cskip=Cskip))
        cur = o2
    st.feat_src = cur
    if net.apply_last_layer:
        K = net.outc.conv.out_channels
        _check_channels(cur.z.shape[3], net.outc.conv)
        y = _empty(N, K, H, W, device=dev)
        L.call("pmu_head1x1_fwd", frame_of([cur.act()], N, H, W), net.outc.conv.weight.data_ptr(),
               L.ptr(net.outc.conv.bias), K, int(net.n_classes == 1), y.data_ptr(), L.stream())
        st.y = y
        return y, st
    C = cur.z.shape[3]
    if cur.z.dtype != F32:
        return frame_to_f32([cur.act()], N, H, W).permute(0, 3, 1, 2), st
    feat = _empty(N, H, W, C, device=dev)
    L.call("pmu_bnrelu_apply", cur.z.data_ptr(), cur.bn.coef.data_ptr(), N * H * W, C, feat.data_ptr(), L.stream())
    return feat.permute(0, 3, 1, 2), st


def unet_backward(net, st: UNetState, dy: torch.Tensor, grads: GradSink | None = None) -> dict:
    """Backward of unet_forward given dL/d(output).  Returns {parameter: grad}."""
    grads = grads if grads is not None else GradSink()
    s = L.stream()
    dev = dy.device
    x = st.x
    N, _, H, W = x.shape
    last = st.feat_src
    if net.apply_last_layer:
        K = net.outc.conv.out_channels
        C = last.z.shape[3]
        dyc = dy.contiguous()
        lb = L.lib()
        head_fuse = (CFG.head_fuse and K <= 8 and last.z.dtype == F32 and last.bn.mean is not None
                     and lb.pmu_head1x1_bwd_bnr_ok(N, H, W, C) and (not last.bf16 or C % 8 == 0))
        dl = None if head_fuse else _empty(N, K, H, W, device=dev)
        da = None if head_fuse else _empty(N, H, W, C, device=dev)
        dwo = grads.new(net.outc.conv.weight)
        dbo = grads.new(net.outc.conv.bias) if net.outc.conv.bias is not None else _empty(K, device=dev)
        wsb = lb.pmu_wgrad1x1_ws(N * H * W, K, C)
        ws = _empty(max(1, (wsb + 3) // 4), device=dev)
        if last.z.dtype == F32 and last.bn.mean is not None and lb.pmu_head1x1_bwd_bnr_ok(N, H, W, C):
            # one pass over z: the head's input gradient, its weight / bias gradient and the last
            # layer's BN-backward partial sums
            R = lb.pmu_head1x1_bwd_tiles(N, H, W)
            part = _empty(R, 2 * C, device=dev)
            L.call("pmu_head1x1_bwd_bnr", dyc.data_ptr(), st.y.data_ptr(), int(net.n_classes == 1),
                   net.outc.conv.weight.data_ptr(), K, C, N, H, W, None, L.ptr(da), last.z.data_ptr(),
                   last.bn.coef.data_ptr(), last.bn.mean.data_ptr(), last.bn.invstd.data_ptr(), part.data_ptr(),
                   dwo.data_ptr(), dbo.data_ptr(), ws.data_ptr(), wsb, s)
            if head_fuse:   # da unstored: the last layer's dz comes from dy (HeadDa)
                da = HeadDa(dyc, st.y, net.n_classes == 1, net.outc.conv.weight, K, last)
            last.bnr = (da, part, R)
        else:
            L.call("pmu_head1x1_bwd", dyc.data_ptr(), st.y.data_ptr(), int(net.n_classes == 1),
                   net.outc.conv.weight.data_ptr(), K, C, N, H, W, dl.data_ptr(), da.data_ptr(), s)
            L.call("pmu_wgrad1x1", dl.data_ptr(), frame_of([last.act()], N, H, W), K, dwo.data_ptr(), dbo.data_ptr(),
                   ws.data_ptr(), wsb, s)
        grads.flush()
    else:
        da = dy.permute(0, 2, 3, 1).contiguous()   # NCHW-shaped channels-last view -> NHWC

    nlev = len(st.enc)
    dskip = [None] * nlev
    # ---- decoder, last block first
    for j in reversed(range(len(net.up_blocks))):
        up = net.up_blocks[j]
        us: UpState = st.ups[j]
        c1w, b1, c2w, b2 = _dc_layers(up.conv)
        da1 = conv_bn_backward(us.c2, da, c2w, b2, grads, dx_bf16=True)
        grads.flush()
        Cskip = us.cskip
        convT = up.up
        prev = us.prev
        hi, wi, Cin_t = prev.z.shape[1], prev.z.shape[2], prev.z.shape[3]
        Cup = convT.out_channels
        # bf16 with the LDS-DMA transposed-conv input gradient and no F.pad: dup is needed only in bf16 and
        # for the bias gradient's column sums, which the concat input gradient forms in its epilogue
        x1only = bool(us.bf16 and us.off == (0, 0) and L.lib().pmu_convT2x2_dma_ok(Cin_t, Cup, 1))
        dsk, dup = conv_bn_backward(us.c1, da1, c1w, b1, grads, split=Cskip, x1_bf16_only=x1only, dx_bf16=True)
        grads.flush()
        dskip[nlev - 2 - j] = dsk
        Hd, Wd = dup.shape[1], dup.shape[2]
        # bf16 dx from the LDS-DMA transposed-conv input gradient (CFG.dx_bf16): its consumer is the next
        # layer's BN backward (pmu_bn_bwd_reduce_dxb, the BN-backward frames)
        dxb = bool(us.bf16 and CFG.dx_bf16 and L.lib().pmu_convT2x2_dma_ok(Cin_t, Cup, 1))
        dx = _empty(N, hi, wi, Cin_t, dtype=BF16S if dxb else F32, device=dev)
        dut = None
        dbpart = getattr(dup, "_pmu_dbpart", None)
        if dbpart is not None:
            dut = dup
        elif us.bf16:   # the concat dgrad's bf16 copy of dup when it wrote one (pmu_conv3x3_dgrad_dma_x1b)
            dut = getattr(dup, "_pmu_bf16", None)
            dut = dut if dut is not None else frame_to_bf16([Src(dup)], N, Hd, Wd)
        if us.bf16 and L.lib().pmu_convT2x2_dma_ok(Cin_t, Cup, 1):
            wpt = pack_convT_weights_dma(convT.weight, dgrad=True)
            L.call("pmu_convT2x2_dgrad_dma_dxb" if dxb else "pmu_convT2x2_dgrad_dma", dut.data_ptr(), dut.shape[3], Hd,
                   Wd, us.off[0], us.off[1], wpt.data_ptr(), N, hi, wi, Cin_t, Cup, dx.data_ptr(), s)
        elif us.bf16 and Cin_t % 128 == 0 and Cup % 32 == 0 and L.experiments_build():
            wpt = pack_convT_weights_bf16(convT.weight, dgrad=True)
            L.call("pmu_convT2x2_dgrad_bf16", dup.data_ptr(), Hd, Wd, us.off[0], us.off[1], wpt.data_ptr(), N, hi, wi,
                   Cin_t, Cup, dx.data_ptr(), s)
        else:
            wpt = pack_convT_weights(convT.weight, dgrad=True)
            L.call("pmu_convT2x2_dgrad", dup.data_ptr(), Hd, Wd, us.off[0], us.off[1], convT.weight.data_ptr(),
                   wpt.data_ptr(), N, hi, wi, Cin_t, Cup, dx.data_ptr(), s)
        dwt = grads.new(convT.weight)
        dbt = grads.new(convT.bias) if convT.bias is not None else None
        if us.bf16:
            # bf16 operands materialised (the convT input after BN+ReLU, du); the bias gradient sums fp32 du
            xt = us.xt if us.xt is not None else frame_to_bf16([prev.act()], N, hi, wi)
            us.xt = None
            wsb = L.lib().pmu_convT2x2_wgrad_ws_bf16(N, hi, wi, Cin_t, Cup)
            ws = _empty(max(1, (wsb + 3) // 4), device=dev)
            if dbpart is not None:
                L.call("pmu_convT2x2_wgrad_bf16", xt.data_ptr(), dut.data_ptr(), None, N, hi, wi, Hd, Wd,
                       0, 0, Cin_t, Cup, dwt.data_ptr(), None, ws.data_ptr(), wsb, s)
                if dbt is not None:
                    part, R, sp = dbpart
                    wsd = _empty(L.lib().pmu_convT2x2_dbias_rows_ws(Cup) // 4, device=dev)
                    L.call("pmu_convT2x2_dbias_rows", part.data_ptr() + 4 * sp, R, part.shape[1], Cup,
                           dbt.data_ptr(), wsd.data_ptr(), s)
            else:
                L.call("pmu_convT2x2_wgrad_bf16", xt.data_ptr(), dut.data_ptr(), dup.data_ptr(), N, hi, wi, Hd, Wd,
                       us.off[0], us.off[1], Cin_t, Cup, dwt.data_ptr(), L.ptr(dbt), ws.data_ptr(), wsb, s)
            del xt, dut
        else:
            wsb = L.lib().pmu_convT2x2_wgrad_ws(N, hi, wi, Cin_t, Cup)
            ws = _empty(max(1, (wsb + 3) // 4), device=dev)
            L.call("pmu_convT2x2_wgrad", dup.data_ptr(), Hd, Wd, us.off[0], us.off[1],
                   frame_of(_f32_srcs([prev.act()], N, hi, wi), N, hi, wi), Cup, dwt.data_ptr(), L.ptr(dbt),
                   ws.data_ptr(), wsb, s)
        grads.flush()
        da = dx
    # ---- encoder, deepest first; da = gradient w.r.t. the deepest encoder output
    for lev in reversed(range(nlev)):
        o1, o2 = st.enc[lev]
        if lev == 0:
            c1w, b1, c2w, b2 = _dc_layers(net.inc)
        else:
            c1w, b1, c2w, b2 = _dc_layers(net.down_blocks[lev - 1].maxpool_conv[1])
        if lev != nlev - 1:
            da = dskip[lev]   # skip grad with the pooled path accumulated below
        da1 = conv_bn_backward(o2, da, c2w, b2, grads, dx_bf16=True)
        grads.flush()
        dpool = conv_bn_backward(o1, da1, c1w, b1, grads, need_dx=(lev > 0), dx_bf16=True)
        grads.flush()
        if lev > 0:
            prev = st.enc[lev - 1][1]
            hp, wp = prev.z.shape[1], prev.z.shape[2]
            Cp = prev.z.shape[3]
            dsk = dskip[lev - 1]
            bn_ok = prev.z.dtype == F32 and prev.bn.mean is not None and Cp % 4 == 0
            if bn_ok and dpool.dtype == BF16S and dsk.dtype == BF16S and CFG.pool_fuse and prev.bf16 \
                    and pool_fuse_ok(Cp):
                # bf16 pooled and skip gradients (*_dxb): the pooled layer's da = their fp32 sum stays
                # unstored (PoolSumDa) — its BN-backward partial sums here, its bf16 dz in that layer's
                # backward
                R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, hp, wp, Cp)
                part = _empty(R, 2 * Cp, device=dev)
                L.call("pmu_maxpool2_bwd_bnr_stats_dxb", dpool.data_ptr(), dsk.data_ptr(), prev.z.data_ptr(),
                       prev.bn.coef.data_ptr(), prev.bn.mean.data_ptr(), prev.bn.invstd.data_ptr(), N, hp, wp, Cp,
                       part.data_ptr(), s)
                dsum = PoolSumDa(dpool, dsk, prev)
                dskip[lev - 1] = dsum
                prev.bnr = (dsum, part, R)
                continue
            if bn_ok and dpool.dtype == BF16S and dsk.dtype == BF16S:
                # bf16 pooled and skip gradients (*_dxb): their fp32 sum is the pooled layer's da, written
                # to a new tensor with that layer's BN-backward partial sums
                R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, hp, wp, Cp)
                part = _empty(R, 2 * Cp, device=dev)
                dsum = _empty(N, hp, wp, Cp, device=dev)
                L.call("pmu_maxpool2_bwd_bnr_dxb", dpool.data_ptr(), dsk.data_ptr(), prev.z.data_ptr(),
                       prev.bn.coef.data_ptr(), prev.bn.mean.data_ptr(), prev.bn.invstd.data_ptr(), N, hp, wp, Cp,
                       dsum.data_ptr(), part.data_ptr(), s)
                dskip[lev - 1] = dsum
                prev.bnr = (dsum, part, R)
                continue
            # (mixed storage: the fp32 kernels below on fp32 copies)
            if dpool.dtype == BF16S:
                dpool = frame_to_f32([Src(dpool)], N, hp // 2, wp // 2)
            if dsk.dtype == BF16S:
                dskip[lev - 1] = frame_to_f32([Src(dsk)], N, hp, wp)
            if bn_ok and CFG.pool_fuse and pool_fuse_ok(Cp) and dpool.dtype == F32 and dskip[lev - 1].dtype == F32:
                # fp32 parts (config c2): the pooled layer's da stays unstored as above (fp32 dz)
                dsk = dskip[lev - 1]
                R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, hp, wp, Cp)
                part = _empty(R, 2 * Cp, device=dev)
                L.call("pmu_maxpool2_bwd_bnr_stats", dpool.data_ptr(), dsk.data_ptr(), prev.z.data_ptr(),
                       prev.bn.coef.data_ptr(), prev.bn.mean.data_ptr(), prev.bn.invstd.data_ptr(), N, hp, wp, Cp,
                       part.data_ptr(), s)
                dsum = PoolSumDa(dpool, dsk, prev)
                dskip[lev - 1] = dsum
                prev.bnr = (dsum, part, R)
                continue
            if bn_ok:
                # routed into the skip gradient, which completes the pooled layer's da: the same pass
                # forms that layer's BN-backward partial sums (no pmu_bn_bwd_reduce for it)
                R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, hp, wp, Cp)
                part = _empty(R, 2 * Cp, device=dev)
                L.call("pmu_maxpool2_bwd_bnr", dpool.data_ptr(), prev.z.data_ptr(), prev.bn.coef.data_ptr(),
                       prev.bn.mean.data_ptr(), prev.bn.invstd.data_ptr(), N, hp, wp, Cp, dskip[lev - 1].data_ptr(),
                       1, part.data_ptr(), s)
                prev.bnr = (dskip[lev - 1], part, R)
            else:
                L.call("pmu_maxpool2_bwd_zb" if prev.z.dtype == BF16S else "pmu_maxpool2_bwd", dpool.data_ptr(),
                       prev.z.data_ptr(), prev.bn.coef.data_ptr(), N, hp, wp, Cp, dskip[lev - 1].data_ptr(), 1, s)
    return grads


def unet_report_order(net) -> list:
    """The parameter groups in the order unet_backward reports them (one GradSink.flush each): the
    head, then per up block (last first) conv2, conv1 and the ConvTranspose2d, then per encoder level
    (deepest first) conv2 and conv1 — within a conv layer BN weight, BN bias, conv bias, conv weight.
    This is the layout pmu_hip.dp learns from the first data-parallel step (and what the CPU tests
    of the bucket logic replay)."""
    def conv_group(conv, bn):
        return [p for p in (bn.weight, bn.bias, conv.bias, conv.weight) if p is not None]
    groups = []
    if net.apply_last_layer:
        groups.append([p for p in (net.outc.conv.weight, net.outc.conv.bias) if p is not None])
    for j in reversed(range(len(net.up_blocks))):
        up = net.up_blocks[j]
        c1w, b1, c2w, b2 = _dc_layers(up.conv)
        groups += [conv_group(c2w, b2), conv_group(c1w, b1),
                   [p for p in (up.up.weight, up.up.bias) if p is not None]]
    blocks = [net.inc] + [d.maxpool_conv[1] for d in net.down_blocks]
    for dc in reversed(blocks):
        c1w, b1, c2w, b2 = _dc_layers(dc)
        groups += [conv_group(c2w, b2), conv_group(c1w, b1)]
    return groups


# ----------------------------------------------------------------------------------------
# packed weights: cached across calls, re-packed in one launch per layout by the optimizer
# ----------------------------------------------------------------------------------------
# A conv's weights are re-laid out (Winograd U = G g G^T, bf16 tiles, ...) for its kernels.  They only
# change in the optimizer step, so each pack is kept and reused until its tensor changes: the entry
# records the parameter's storage, torch's in-place version counter and a pack epoch that
# pmu_hip.optim.FusedSGD bumps (its kernel writes the parameters through raw pointers, which torch's
# version counter does not see).  After its update FusedSGD calls repack(), which refreshes every
# cached pack of the updated parameters in one batched launch per layout (pmu_*_pack_*_multi): the
# forward and backward then launch no pack kernel.  (Writes through ``param.data`` bypass the version
# counter: call invalidate_packs() after them.)
class _Pack:
    __slots__ = ("w", "ptr", "ver", "epoch", "t")


_PACKS: dict = {}
_TABLES: dict = {}
# layout -> (single-tensor packer, batched-launch C entries (blocks query, multi launch))
_LAYOUTS = {
    "dma": (_pack_weights_dma_now, ("pmu_conv3x3_pack_dma_blocks", "pmu_conv3x3_pack_dma_multi")),
    "wino4": (_pack_weights_wino4_now, ("pmu_conv3x3_pack_wino4_blocks", "pmu_conv3x3_pack_wino4_multi")),
    "wino2h": (_pack_weights_wino2h_now, ("pmu_conv3x3_pack_wino2h_blocks", "pmu_conv3x3_pack_wino2h_multi")),
    "convT_dma": (_pack_convT_weights_dma_now, ("pmu_convT2x2_pack_dma_blocks", "pmu_convT2x2_pack_dma_multi")),
    "convT": (_pack_convT_weights_now, ("pmu_convT2x2_pack_blocks", "pmu_convT2x2_pack_multi")),
}


def _cached_pack(layout: str, w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    key = (id(w), layout, bool(dgrad))
    e = _PACKS.get(key)
    ep = getattr(w, "_pmu_epoch", 0)
    if e is not None and e.w() is w and e.ptr == w.data_ptr() and e.ver == w._version and e.epoch == ep:
        return e.t
    e = _Pack()
    e.w = weakref.ref(w, lambda _r, k=key: _PACKS.pop(k, None))
    e.ptr, e.ver, e.epoch = w.data_ptr(), w._version, ep
    e.t = _LAYOUTS[layout][0](w, dgrad)
    _PACKS[key] = e
    return e.t


def invalidate_packs() -> None:
    """Forget every cached pack (after writing parameters through ``.data``)."""
    _PACKS.clear()
    _TABLES.clear()


def repack(params) -> int:
    """After an optimizer step that wrote ``params`` in place: bump their pack epoch and refresh all
    their cached packs, one batched launch per (layout, direction).  Returns the launch count."""
    ids = set()
    for p in params:
        p._pmu_epoch = getattr(p, "_pmu_epoch", 0) + 1
        ids.add(id(p))
    groups = {}
    for key, e in list(_PACKS.items()):
        w = e.w()
        if w is None or id(w) not in ids or e.ptr != w.data_ptr() or e.ver != w._version:
            continue   # not updated here, or changed elsewhere: re-packed on its next use
        groups.setdefault((key[1], key[2]), []).append((w, e))
    launches = 0
    s = L.stream()
    lb = L.lib()
    for (layout, dgrad), items in groups.items():
        blocks_fn, multi = _LAYOUTS[layout][1]
        sig = tuple((w.data_ptr(), e.t.data_ptr(), w.shape[0], w.shape[1]) for w, e in items)
        tab = _TABLES.get((layout, dgrad, sig))
        if tab is None:
            jobs = (L.PmuPackJob * len(items))()
            b0 = 0
            for i, (w, e) in enumerate(items):
                nb = getattr(lb, blocks_fn)(w.shape[0], w.shape[1], int(dgrad))
                jobs[i] = L.PmuPackJob(w.data_ptr(), e.t.data_ptr(), w.shape[0], w.shape[1], b0, nb)
                b0 += nb
            dev_jobs = torch.frombuffer(bytearray(jobs), dtype=torch.uint8).to(items[0][0].device)
            tab = (dev_jobs, len(items), b0)
            if len(_TABLES) > 64:
                _TABLES.clear()
            _TABLES[(layout, dgrad, sig)] = tab
        L.call(multi, tab[0].data_ptr(), tab[1], tab[2], int(dgrad), s)
        launches += 1
        for w, e in items:
            e.epoch = w._pmu_epoch
    return launches


def pack_weights_dma(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """Weights rounded to bf16 in the LDS-DMA conv's swizzled unit order (cached; pmu_conv3x3_pack_dma)."""
    return _cached_pack("dma", w, dgrad)


def pack_weights_wino4(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """F(4x4,3x3) weights U = G g G^T in the F(4x4) kernel's blocks (cached; pmu_conv3x3_pack_wino4)."""
    return _cached_pack("wino4", w, dgrad)


def pack_weights_wino2h(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """F(2x2,3x3) weights in the 1024-thread kernel's 64-channel blocks (cached; pmu_conv3x3_pack_wino2h)."""
    return _cached_pack("wino2h", w, dgrad)


def pack_convT_weights_dma(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """ConvT weights rounded to bf16 in the LDS-DMA GEMMs' unit order (cached; pmu_convT2x2_pack_dma)."""
    return _cached_pack("convT_dma", w, dgrad)


def pack_convT_weights(w: torch.Tensor, dgrad: bool) -> torch.Tensor:
    """ConvT weights [Cin][Cout][2][2] k-contiguous for the pipelined GEMMs (cached; pmu_convT2x2_pack)."""
    return _cached_pack("convT", w, dgrad)
