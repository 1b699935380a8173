"""Three-view volume fusion on the HIP path (row a14): PMU/eval.py:157-203.

The reference concatenates per-slice softmax outputs per view, permutes views 1 and 2 into the
view-0 frame (permute(2,1,0,3) / permute(2,1,3,0)), averages the three volumes, and scores each
of the four volumes with per-class Dice of the argmax one-hot (eval.py:42-49).  Here the per-view
stacks are written by the predictor straight into their final buffers and ONE kernel
(pmu_fuse3view) reads each prediction once: softmax (optional), transposition, average, argmax
label map and exact Dice counts for all four volumes.
"""
from __future__ import annotations

import torch

from . import _lib as L
from .metrics import dice_from_counts

VOLUMES = ("view0", "view1", "view2", "average")


def fuse_views(v0: torch.Tensor, v1: torch.Tensor, v2: torch.Tensor, truth: torch.Tensor, logits: bool = False,
               want_avg: bool = True, want_label: bool = True) -> dict:
    """v0 (D0,C,D1,D2), v1 (D1,C,D0,D2), v2 (D2,C,D0,D1) per-view stacks; truth (D0,D1,D2) labels.

    Returns {'avg': (D0,C,D1,D2) or None, 'label': (D0,D1,D2) int32 or None,
             'counts': (4,C,3) float64, 'dice': (4,C) float32} — dice[v][c] is eval.py's
    dice(volume_v, truth, c) for v in VOLUMES."""
    for t in (v0, v1, v2, truth):
        if not t.is_cuda:
            raise RuntimeError("fuse_views runs on the MI355X HIP path only (there is no CPU fallback)")
    D0, C, D1, D2 = v0.shape
    if tuple(v1.shape) != (D1, C, D0, D2) or tuple(v2.shape) != (D2, C, D0, D1):
        raise ValueError(f"view stacks do not describe one volume: {tuple(v0.shape)}, {tuple(v1.shape)}, "
                         f"{tuple(v2.shape)}")
    dev = v0.device
    tr = truth.reshape(D0, D1, D2).float().contiguous()
    a = [t.float().contiguous() for t in (v0, v1, v2)]
    avg = torch.empty(D0, C, D1, D2, dtype=torch.float32, device=dev) if want_avg else None
    label = torch.empty(D0, D1, D2, dtype=torch.int32, device=dev) if want_label else None
    counts = torch.empty(4, C, 3, dtype=torch.float64, device=dev)
    L.call("pmu_fuse3view", a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(), tr.data_ptr(), D0, D1, D2, C,
           int(bool(logits)), L.ptr(avg), L.ptr(label), counts.data_ptr(), L.stream())
    return {"avg": avg, "label": label, "counts": counts, "dice": dice_from_counts(counts)}
