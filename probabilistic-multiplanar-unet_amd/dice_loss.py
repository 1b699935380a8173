"""Dice coefficient — drop-in for PMU/dice_loss.py:5-12.

``dice_coeff(pred, target)`` = (2 * sum(pred*target) + 1e-6) / (sum(pred) + sum(target) + 1e-6)
over the whole batch, evaluated from the three sums produced by one HIP reduction
(pmu_dice_sums, fp64 accumulation) and the reference's fp32 ratio.  For 0/1 inputs (the only
way the reference's trainers and eval call it) the sums are exact, so the result is
bit-identical.  The trainers' per-class Dice goes through the fused argmax kernel instead
(pmu_hip.metrics).  GPU tensors only: there is no CPU fallback.
"""
import torch

from pmu_hip import _lib as L
from pmu_hip.metrics import SMOOTH


def dice_coeff(pred, target):
    if not (isinstance(pred, torch.Tensor) and isinstance(target, torch.Tensor) and pred.is_cuda and target.is_cuda):
        raise RuntimeError("dice_coeff runs on the MI355X HIP path only: pass GPU tensors (there is no CPU fallback)")
    num = pred.size(0)
    a = pred.reshape(num, -1).float().contiguous()
    b = target.reshape(num, -1).float().contiguous()
    if a.numel() != b.numel():
        raise RuntimeError(f"dice_coeff: pred has {a.numel()} elements, target {b.numel()}")
    sums = torch.empty(3, dtype=torch.float64, device=pred.device)
    L.call("pmu_dice_sums", a.data_ptr(), b.data_ptr(), a.numel(), sums.data_ptr(), L.stream())
    s = sums.float()
    return (2.0 * s[0] + SMOOTH) / (s[1] + s[2] + SMOOTH)
