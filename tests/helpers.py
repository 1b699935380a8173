"""Shared comparison helpers for parity tests (tolerances from SURVEY.md §4)."""
import torch

ACT_TOL = 1e-3    # forward activations / outputs, absolute
LOSS_RTOL = 1e-3  # losses, relative
GRAD_TOL = 1e-3   # gradients: max |dg| / max |g_ref| over the tensor set (globally normalised)


def max_abs(a, b):
    return float((a.detach().double().cpu() - b.detach().double().cpu()).abs().max())


def grad_err(got: dict, ref: dict):
    """Globally normalised max-abs gradient error and the worst key."""
    gmax = max(float(v.abs().max()) for v in ref.values())
    worst, wk = 0.0, None
    for k, r in ref.items():
        e = max_abs(got[k], r) / gmax
        if e > worst:
            worst, wk = e, k
    return worst, wk
