"""CPU oracle for the data-side rows: the multi-planar slicer (a13) and 3-view fusion (a14).

TEST INFRASTRUCTURE ONLY (same rules as oracle/unet_ref.py).  Restated from scratch in numpy /
torch-CPU (PMU/ = /root/reference/Probabilistic-Multiplanar-Unet/):
  * slicer: PMU/utils/mri_dataset.py:11-143 — pinned by tests/golden/g5_slicer.npz (produced by
    importing the reference with in-memory volumes);
  * fusion: PMU/eval.py:42-65,157-203 — the script itself does not parse (:137-138); G6 is
    produced by executing the reference's own ``dice`` and ``slices_to_volume`` helpers (:42-65)
    on the restated main-block flow (tests/golden/make_golden.py g6).
"""
from __future__ import annotations

import numpy as np
import torch


# ----------------------------------------------------------------------------- slicer
def pad_dimensions(vol):
    """Zeros appended to the end of the (first) argmin axis, up to the max dim (:85-98)."""
    diff = max(vol.shape) - min(vol.shape)
    if diff == 0:
        return vol
    ax = int(np.argmin(vol.shape))
    pad = [(0, 0)] * 3
    pad[ax] = (0, diff)
    return np.pad(vol, pad)


def sample_slice(vol, view, i):
    """view 0/1/2 = vol[i,:,:] / vol[:,i,:] / vol[:,:,i] (:70-82)."""
    return [vol[i, :, :], vol[:, i, :], vol[:, :, i]][view]


def preprocess(sl, label=False):
    """(H,W) -> (1,H,W); image / its max when the max is non-zero (:101-112)."""
    out = sl[None, :, :]
    if not label and np.max(out) != 0:
        out = out / np.max(out)
    return out


def build_dataset(scans, filt=True):
    """scans: list of (image, mask) arrays in listdir order.  Returns (image_dims, index_map, items)
    with items[i] = (image f32 (1,H,W), mask f32 (1,H,W)) as MRI_Dataset.__getitem__ (:117-142)."""
    image_dims = tuple([int(np.max(scans[0][0].shape))] * scans[0][0].ndim)
    index_map = []
    padded = [(pad_dimensions(im), pad_dimensions(mk)) for im, mk in scans]
    for s, (_, mk) in enumerate(padded):
        for v in range(3):
            for i in range(mk.shape[v]):
                if not filt or np.max(sample_slice(mk, v, i)) > 0:
                    index_map.append((s, v, i))
    items = []
    for s, v, i in index_map:
        im, mk = padded[s]
        items.append((preprocess(sample_slice(im, v, i)).astype(np.float32),
                      preprocess(sample_slice(mk, v, i), label=True).astype(np.float32)))
    return image_dims, index_map, items


# ----------------------------------------------------------------------------- fusion
def dice_coeff(pred, target):
    """PMU/dice_loss.py:5-12."""
    num = pred.size(0)
    m1, m2 = pred.reshape(num, -1), target.reshape(num, -1)
    return (2. * (m1 * m2).sum() + 0.000001) / (m1.sum() + m2.sum() + 0.000001)


def class_dice(volume, truth, k):
    """eval.py:42-49: Dice of class k of the argmax one-hot of volume (D0,C,D1,D2) vs truth == k."""
    idx = torch.argmax(volume, 1, keepdim=True)
    one_hot = torch.zeros(volume.shape).scatter_(1, idx, 1)
    return float(dice_coeff(one_hot[:, k], (truth == k).float().squeeze(1)))


def fuse(stack0, stack1, stack2):
    """Per-view stacks (D0,C,D1,D2), (D1,C,D0,D2), (D2,C,D0,D1) -> the three volumes in the view-0
    frame (eval.py:176-188 permutes) and their average (:193)."""
    v1 = stack0
    v2 = stack1.permute(2, 1, 0, 3)
    v3 = stack2.permute(2, 1, 3, 0)
    return v1, v2, v3, (v1 + v2 + v3) / 3.0
