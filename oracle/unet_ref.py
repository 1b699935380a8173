"""CPU oracle: functional restatement of the reference U-Net / Probabilistic U-Net math.

TEST INFRASTRUCTURE ONLY.  Nothing under pmu_hip/, model/, trainer/ or the drivers imports
this module; only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg do.
It is written from scratch on torch CPU functional ops and operates on a state_dict (the
reference's key names), so it needs neither the reference code nor the HIP library.

Parity is pinned: tests/test_cpu_host.py (G1, G2, G4) and tests/test_train_cpu.py (G8, through
oracle/train_ref.py) check this module against golden vectors that tests/golden/make_golden.py
produced by importing the reference itself
(PMU/ = /root/reference/Probabilistic-Multiplanar-Unet/).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _bn(x, sd, pre, training, momentum=0.1, eps=1e-5):
    """BatchNorm2d (PMU/model/unet/unet_parts.py:16,19): batch stats in training, running stats in eval.
    Running stats in ``sd`` are updated in place (unbiased var, momentum 0.1)."""
    rm, rv = sd[pre + "running_mean"], sd[pre + "running_var"]
    y = F.batch_norm(x, rm, rv, sd[pre + "weight"], sd[pre + "bias"], training, momentum, eps)
    if training and (pre + "num_batches_tracked") in sd:
        sd[pre + "num_batches_tracked"] += 1
    return y


def _rb(t):
    return t.to(torch.bfloat16).to(t.dtype)


# torch.autocast(bfloat16) returns a conv's output in bf16.  BF16_Z models the HIP path's storage of
# it (include/pmunet_hip.h pmu_conv3x3_fwd_dma_zb, engine CFG.bf16_z): the convs that run on the
# LDS-DMA kernel (maps >= 32 wide, padded Cin % 16 == 0, Cout % 8 == 0) keep z as bf16(z - rm) + rm,
# rm the BN running mean before the step's update (straight-through gradient).  False: fp32 z.
BF16_Z = False


def _dma_zb(x, cin, cout):
    return BF16_Z and x.shape[3] >= 32 and ((cin + 7) // 8 * 8) % 16 == 0 and cout % 8 == 0


# torch.autocast(bfloat16)'s conv backward returns the input gradient in bf16.  BF16_DX models the HIP
# path's storage of it (include/pmunet_hip.h *_dxb entries, engine CFG.dx_bf16, on by default): the
# convs whose input gradient runs on the LDS-DMA kernel (maps >= 32 wide, pad8(Cout) % 16 == 0,
# Cin % 8 == 0, a concat split on a 32-channel boundary) and the transposed convs whose input gradient
# does (Cin % 128 == 0, Cout % 32 == 0) round dx to bf16 once (RNE), and everything
# downstream (BN backward, max-pool routing, the skip-gradient sum in fp32, the transposed conv's
# input gradient and bias gradient) sees the rounded values.  False: fp32 dx (PMU_DX_BF16=0).
BF16_DX = True


# AUTOCAST_ALL: torch.autocast(bfloat16)'s own semantics instead of the HIP path's shape rules — every
# conv and transposed conv (the Cin <= 4 first layer included) rounds its operands, weights, incoming
# gradient and input gradient to bf16, whatever its shape.  Used to measure what autocast itself does to
# the reference's trajectory (tools/dice_gap_seeds.py) and how far the HIP path's fp32 exceptions (the
# first layer, input gradients of maps < 32 wide, ConvT shapes off the LDS-DMA kernel) sit from it.
AUTOCAST_ALL = False
# Which halves of the bf16 arithmetic Bf16Conv3x3 / Bf16ConvT2x2 apply (attribution experiments,
# tools/dice_gap_seeds.py): "fwd" rounds the forward's operand and weights, "bwd" the backward's dy,
# weights, saved operand and dx.  Both by default (the autocast / HIP arithmetic).
ROUND_PARTS = ("fwd", "bwd")


def _dma_dxb(x, cin, cout, split):
    if AUTOCAST_ALL:
        return BF16_DX
    return (BF16_DX and x.shape[3] >= 32 and ((cout + 7) // 8 * 8) % 16 == 0 and cin % 8 == 0
            and (split is None or split == cin or split % 32 == 0))


def _round_centered(y, off):
    """bf16(y - off) + off per channel, gradient passed straight through (autocast's cast)."""
    o = off.to(y.dtype).view(1, -1, 1, 1)
    return y + (_rb(y - o) + o - y).detach()


class Bf16Conv3x3(torch.autograd.Function):
    """conv3x3(pad 1) with torch.autocast(bfloat16) arithmetic as the HIP bf16 kernels implement it
    (include/pmunet_hip.h, bf16 section): the operand x and the weights are rounded to bf16, the
    exact products summed in the ambient dtype; backward rounds the incoming gradient dy to bf16
    once and forms dx = conv2d_input(rb(w), rb(dy)), dw = conv2d_weight(rb(x), rb(dy)), db = sum dy; with
    ``round_dx`` (BF16_DX, the HIP path's *_dxb input gradient) dx itself is rounded to bf16 once."""

    @staticmethod
    def forward(ctx, x, w, b, round_dx=False):
        xr, wr = _rb(x), _rb(w)
        ctx.save_for_backward(xr if "bwd" in ROUND_PARTS else x, wr if "bwd" in ROUND_PARTS else w)
        ctx.has_b = b is not None
        ctx.round_dx = round_dx and "bwd" in ROUND_PARTS
        ctx.rdy = "bwd" in ROUND_PARTS
        if "fwd" not in ROUND_PARTS:
            return F.conv2d(x, w, b, padding=1)
        return F.conv2d(xr, wr, b, padding=1)

    @staticmethod
    def backward(ctx, dy):
        xr, wr = ctx.saved_tensors
        dyr = _rb(dy) if ctx.rdy else dy
        dx = torch.nn.grad.conv2d_input(xr.shape, wr, dyr, padding=1)
        if ctx.round_dx:
            dx = _rb(dx)
        dw = torch.nn.grad.conv2d_weight(xr, wr.shape, dyr, padding=1)
        db = dy.sum((0, 2, 3)) if ctx.has_b else None
        return dx, dw, db, None


class Bf16ConvT2x2(torch.autograd.Function):
    """ConvTranspose2d(k2, s2) with the HIP bf16 path's arithmetic: the forward rounds the operand
    and the weights to bf16 (when ``fwd``), the input gradient rounds dy and the weights (when
    ``dgrad``); the weight gradient multiplies the rounded input and dy (pmu_convT2x2_wgrad_bf16),
    the bias gradient sums the unrounded dy."""

    @staticmethod
    def forward(ctx, x, w, b, fwd, dgrad, round_dx=False):
        ctx.save_for_backward(x, w)
        bwd = "bwd" in ROUND_PARTS
        ctx.dgrad, ctx.has_b, ctx.round_dx, ctx.rw = dgrad and bwd, b is not None, round_dx and bwd, bwd
        fwd = fwd and "fwd" in ROUND_PARTS
        return F.conv_transpose2d(_rb(x) if fwd else x, _rb(w) if fwd else w, b, stride=2)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = F.conv2d(_rb(dy) if ctx.dgrad else dy, _rb(w) if ctx.dgrad else w, stride=2)
        if ctx.round_dx:   # BF16_DX: pmu_convT2x2_dgrad_dma_dxb stores dx in bf16
            dx = _rb(dx)
        n, k = dy.shape[0], dy.shape[1]
        rb = _rb if ctx.rw else (lambda t: t)
        dw = torch.einsum("ncij,nkiajb->ckab", rb(x), rb(dy).reshape(n, k, x.shape[2], 2, x.shape[3], 2))
        db = dy.sum((0, 2, 3)) if ctx.has_b else None
        return dx, dw, db, None, None, None


def _conv3x3(x, w, b, bf16, round_dx=False):
    return Bf16Conv3x3.apply(x, w, b, round_dx) if bf16 else F.conv2d(x, w, b, padding=1)


def double_conv(x, sd, pre, training, bf16=False, first_fp32=False, split=None, dxb=False):
    """(conv3x3 pad1 -> BN -> ReLU) x 2  (unet_parts.py:14-21); Sequential indices 0,1,3,4.
    bf16: the autocast arithmetic of Bf16Conv3x3 (first_fp32 keeps the first conv in fp32, as the
    HIP path's Cin <= 4 first-layer kernel).  dxb: the block sits inside the UNet's backward, where the
    HIP path keeps bf16 activation gradients (BF16_DX); split: the first conv's concat split."""
    for i in (0, 3):
        use = bf16 and (AUTOCAST_ALL or not (first_fp32 and i == 0))
        w = sd[f"{pre}double_conv.{i}.weight"]
        zb = use and _dma_zb(x, w.shape[1], w.shape[0])
        rdx = use and dxb and _dma_dxb(x, w.shape[1], w.shape[0], split if i == 0 else None)
        x = _conv3x3(x, w, sd[f"{pre}double_conv.{i}.bias"], use, rdx)
        if zb:
            x = _round_centered(x, sd[f"{pre}double_conv.{i + 1}.running_mean"].clone())
        x = F.relu(_bn(x, sd, f"{pre}double_conv.{i + 1}.", training))
    return x


def unet_forward(sd, x, n_levels, n_classes, apply_last_layer=True, training=True, bf16=False):
    """UNet.forward (PMU/model/unet/unet_model.py:31-54).

    n_levels = len(num_filters).  Down_i = MaxPool2d(2) + DoubleConv (unet_parts.py:31-34);
    Up = ConvTranspose2d(k2,s2) -> F.pad to the skip size -> cat([skip, up]) -> DoubleConv
    (unet_parts.py:52,58-66); up_blocks stored deepest-first (unet_model.py:29); skip of up
    block i is xs[-(2 + 2i)] (:39).  bf16: every 3x3 conv but a Cin <= 4 first one in Bf16Conv3x3
    arithmetic (the HIP path's autocast mode)."""
    xs = [double_conv(x, sd, "inc.", training, bf16, first_fp32=x.shape[1] <= 4, dxb=True)]
    for i in range(n_levels - 1):
        xs.append(double_conv(F.max_pool2d(xs[-1], 2), sd, f"down_blocks.{i}.maxpool_conv.1.", training, bf16,
                              dxb=True))
    for i in range(n_levels - 1):
        x1, x2 = xs[-1], xs[-(2 + 2 * i)]
        pre = f"up_blocks.{i}."
        wt = sd[pre + "up.weight"]
        if bf16:  # the HIP path's bf16 convT where its kernels take the shapes (pmu_convT2x2_bf16_ok)
            cin, cout = wt.shape[0], wt.shape[1]
            fwd_b = AUTOCAST_ALL or (cin % 32 == 0 and cout % 32 == 0 and (4 * cout) % 128 == 0)
            dma_d = AUTOCAST_ALL or (cin % 128 == 0 and cout % 32 == 0)   # pmu_convT2x2_dma_ok(cin, cout, 1)
            x1 = Bf16ConvT2x2.apply(x1, wt, sd[pre + "up.bias"], fwd_b, dma_d, BF16_DX and dma_d)
        else:
            x1 = F.conv_transpose2d(x1, wt, sd[pre + "up.bias"], stride=2)
        dy, dx = x2.shape[2] - x1.shape[2], x2.shape[3] - x1.shape[3]
        x1 = F.pad(x1, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2])
        xs.append(double_conv(torch.cat([x2, x1], dim=1), sd, pre + "conv.", training, bf16, split=x2.shape[1],
                              dxb=True))
    feat = xs[-1]
    if not apply_last_layer:
        return feat
    out = F.conv2d(feat, sd["outc.conv.weight"], sd["outc.conv.bias"])
    if n_classes == 1:
        out = torch.sigmoid(out)
    return out


def unet_loss(out, target, n_classes):
    """UNetTrainer.loss (PMU/trainer/unet_trainer.py:23,30-37): BCELoss(mean) on sigmoid
    output for 1 class, CrossEntropyLoss(mean) with target.squeeze(1) otherwise."""
    if n_classes == 1:
        return F.binary_cross_entropy(out, target)
    return F.cross_entropy(out, target.squeeze(1).long())


def sgd_clip_step(params, grads, bufs, lr, momentum=0.9, clip=0.1):
    """clip_grad_value_(0.1) + SGD(momentum, dampening 0) (PMU/train.py:65,108-110); bufs start at 0."""
    for k in params:
        g = grads[k].clamp(-clip, clip)
        bufs[k] = momentum * bufs[k] + g
        params[k] = params[k] - lr * bufs[k]


def dice_coeff(pred, target):
    """PMU/dice_loss.py:5-12: whole-batch Dice with smooth 1e-6."""
    smooth = 0.000001
    num = pred.size(0)
    m1 = pred.reshape(num, -1)
    m2 = target.reshape(num, -1)
    inter = (m1 * m2).sum()
    return (2. * inter + smooth) / (m1.sum() + m2.sum() + smooth)


def trainer_dice(masks_pred, true_masks, n_classes):
    """UNetTrainer.eval / ProbUNetTrainer.eval (unet_trainer.py:39-58): per-class Dice of the
    softmax-argmax one-hot prediction (classes >= 1), or (pred > 0.5) for 1 class."""
    if n_classes == 1:
        return [float(dice_coeff((masks_pred > 0.5).float(), true_masks))]
    probs = F.softmax(masks_pred, dim=1)
    idx = torch.argmax(probs, 1, keepdim=True)
    one_hot = torch.zeros_like(probs).scatter_(1, idx, 1)
    return [float(dice_coeff(one_hot[:, k], (true_masks == k).float().squeeze(1)))
            for k in range(1, one_hot.shape[1])]


def unet_param_keys(sd):
    """Trainable parameter keys of a U-Net state_dict in module registration order."""
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                  or k.endswith("num_batches_tracked"))]


def unet_train_step(sd, x, target, n_levels, n_classes, lr=None, bufs=None, bf16=False):
    """One reference training step on CPU: forward, loss, backward (+ optional clip/SGD).
    Returns (out, loss, grads) and updates sd's running stats (and params if lr).  bf16: the forward in
    the HIP path's torch.autocast(bfloat16) arithmetic (unet_forward's bf16)."""
    keys = unet_param_keys(sd)
    params = {k: sd[k].detach().clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    out = unet_forward(work, x, n_levels, n_classes, bf16=bf16)
    loss = unet_loss(out, target, n_classes)
    loss.backward()
    grads = {k: params[k].grad.detach().clone() for k in keys}
    for k in sd:
        if k not in params:
            sd[k] = work[k]
    if lr is not None:
        cur = {k: sd[k].detach() for k in keys}
        sgd_clip_step(cur, grads, bufs, lr)
        for k in keys:
            sd[k] = cur[k]
    return out.detach(), loss.detach(), grads
