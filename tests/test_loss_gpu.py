"""GPU parity of the HIP losses (row a6) with torch's CPU criteria on the same inputs: nn.BCELoss on
probabilities (incl. exact 0 / 1 values: the -100 log clamp) and nn.CrossEntropyLoss on logits
(incl. ignore_index), every reduction, value and input gradient (PMU/trainer/unet_trainer.py:23,
30-37; probabilistic_unet.py:286-304).  Tolerance: rel 1e-5 on values, 1e-5 of max|g| on grads."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _close(a, b, tol=1e-5):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) <= tol * max(1.0, float(b.abs().max()))


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_bce_loss(dev, reduction):
    from pmu_hip.loss import BCELoss
    g = torch.Generator().manual_seed(1)
    y = torch.rand(4, 1, 33, 29, generator=g)
    y[0, 0, 0, :5] = torch.tensor([0.0, 1.0, 1e-30, 1 - 1e-7, 0.5])
    t = (torch.rand(4, 1, 33, 29, generator=g) > 0.5).float()
    yr = y.clone().requires_grad_(True)
    ref = nn.BCELoss(reduction=reduction)(yr, t)
    yd = y.to(dev).requires_grad_(True)
    got = BCELoss(reduction=reduction)(yd, t.to(dev))
    assert got.shape == ref.shape and _close(got, ref)
    w = torch.rand(ref.shape, generator=g) if reduction == "none" else torch.tensor(0.7)
    (ref * w).sum().backward()
    (got * w.to(dev)).sum().backward()
    mask = torch.ones_like(y, dtype=torch.bool)
    mask[0, 0, 0, :3] = False          # y in {0, 1}: both sides divide by the 1e-12 floor (~1e12 grads)
    assert _close(yd.grad.cpu()[mask], yr.grad[mask])
    assert torch.isfinite(yd.grad).all()


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
@pytest.mark.parametrize("K", [2, 3, 5])
def test_cross_entropy_loss(dev, reduction, K):
    from pmu_hip.loss import CrossEntropyLoss
    g = torch.Generator().manual_seed(K)
    x = torch.randn(3, K, 21, 17, generator=g) * 3
    t = torch.randint(0, K, (3, 21, 17), generator=g)
    t[1, 2, :6] = -100                 # ignore_index
    xr = x.clone().requires_grad_(True)
    ref = nn.CrossEntropyLoss(reduction=reduction)(xr, t)
    xd = x.to(dev).requires_grad_(True)
    got = CrossEntropyLoss(reduction=reduction)(xd, t.to(dev))
    assert got.shape == ref.shape and _close(got, ref)
    w = torch.rand(ref.shape, generator=g) if reduction == "none" else torch.tensor(1.3)
    (ref * w).sum().backward()
    (got * w.to(dev)).sum().backward()
    assert _close(xd.grad, xr.grad)


def test_losses_refuse_cpu_and_unused_options():
    from pmu_hip.loss import BCELoss, CrossEntropyLoss
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        BCELoss()(torch.rand(2, 2), torch.rand(2, 2))
    with pytest.raises(NotImplementedError):
        CrossEntropyLoss(label_smoothing=0.1)(torch.rand(2, 3), torch.zeros(2, dtype=torch.long))


def test_cross_entropy_out_of_range_target_is_loud(dev):
    """A class target outside [0, K) that is not ignore_index: torch raises; the HIP loss (no host
    synchronisation on the hot path) returns NaN for the loss and that pixel's gradient, and the
    bounds-checked debug build records the index (pmu_debug_read)."""
    from pmu_hip import _lib as L
    from pmu_hip.loss import CrossEntropyLoss
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 3, 8, 8, generator=g)
    t = torch.randint(0, 3, (2, 8, 8), generator=g)
    t[0, 0, 0] = 3
    with pytest.raises(IndexError):
        nn.CrossEntropyLoss()(x, t)
    xd = x.to(dev).requires_grad_(True)
    got = CrossEntropyLoss()(xd, t.to(dev))
    got.backward()
    assert torch.isnan(got).item()
    assert torch.isnan(xd.grad[0, :, 0, 0]).all() and torch.isfinite(xd.grad[1]).all()
    if L.debug_build():
        with pytest.raises(RuntimeError, match="index out of range"):
            L.debug_check()
