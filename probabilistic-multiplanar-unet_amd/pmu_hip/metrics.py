"""Dice on the HIP path (row a8): PMU/dice_loss.py:5-12 and the trainers' eval()
(PMU/trainer/unet_trainer.py:39-58, probunet_trainer.py:41-60).

One kernel (pmu_dice_counts) produces exact integer counts (intersection, |pred|, |target|) per
class straight from the logits/probabilities: threshold (1 class) or softmax-argmax one-hot
(several classes, first maximum like torch.argmax), so no one-hot tensor is materialised.  The
final ratio is evaluated in fp32 exactly as the reference does with its fp32 sums (counts below
2^24 are exact in fp32, so the result is bit-identical).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

SMOOTH = 0.000001   # dice_loss.py:6


def dice_counts(y: torch.Tensor, mask: torch.Tensor, n_classes: int) -> torch.Tensor:
    """(K, 3) float64 counts on the device; y (N,K,H,W), mask (N,1,H,W) or (N,H,W)."""
    if not y.is_cuda:
        raise RuntimeError("dice_counts runs on the MI355X HIP path only (there is no CPU fallback)")
    N, K, H, W = y.shape
    if K != n_classes:
        raise ValueError(f"prediction has {K} channels, expected n_classes={n_classes}")
    yc = y.detach().float().contiguous()
    mc = mask.detach().to(device=y.device, dtype=torch.float32).reshape(N, H, W).contiguous()
    counts = torch.empty(K, 3, dtype=torch.float64, device=y.device)
    L.call("pmu_dice_counts", yc.data_ptr(), mc.data_ptr(), N, K, H, W, counts.data_ptr(), L.stream())
    return counts


def dice_counts_many(ys: torch.Tensor, mask: torch.Tensor, n_classes: int) -> torch.Tensor:
    """(S, K, 3) float64 counts of S predictions ys (S,N,K,H,W) against one mask, in one launch
    (pmu_dice_counts_many) — the same integers as S dice_counts calls (the trainers' eval over
    several samples, probunet_trainer.py:41-60)."""
    if not ys.is_cuda:
        raise RuntimeError("dice_counts runs on the MI355X HIP path only (there is no CPU fallback)")
    S, N, K, H, W = ys.shape
    if K != n_classes:
        raise ValueError(f"prediction has {K} channels, expected n_classes={n_classes}")
    yc = ys.detach().float().contiguous()
    mc = mask.detach().to(device=ys.device, dtype=torch.float32).reshape(N, H, W).contiguous()
    counts = torch.empty(S, K, 3, dtype=torch.float64, device=ys.device)
    L.call("pmu_dice_counts_many", yc.data_ptr(), mc.data_ptr(), S, N, K, H, W, counts.data_ptr(), L.stream())
    return counts


def dice_from_counts(c: torch.Tensor) -> torch.Tensor:
    """fp32 (2 I + s) / (P + T + s), the reference's arithmetic on its fp32 sums."""
    c = c.float()
    return (2.0 * c[..., 0] + SMOOTH) / (c[..., 1] + c[..., 2] + SMOOTH)


def trainer_dice(masks_pred: torch.Tensor, true_masks: torch.Tensor, n_classes: int) -> np.ndarray:
    """The trainers' eval(): [dice] for 1 class (pred > 0.5), else Dice of classes 1..K-1."""
    d = dice_from_counts(dice_counts(masks_pred, true_masks, n_classes)).cpu().numpy().astype(np.float64)
    return d[:1] if n_classes == 1 else d[1:]
