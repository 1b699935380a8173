"""CPU checks of the data-side rows and the DP host logic: slicer oracle vs the reference's G5,
fusion restatement vs G6, the oracle's gradient accumulation vs the reference's G7, micro-batch
dealing of train.py's data-parallel loop, and CPU refusal of the GPU-only drop-ins."""
import os

import numpy as np
import pytest
import torch

from helpers import grad_err, max_abs

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def g5_scans(z):
    names = sorted({k.split("/")[1] for k in z.files if k.startswith("vol/")})
    return names, [(z[f"vol/{n}/img"], z[f"vol/{n}/lab"]) for n in names]


@pytest.mark.parametrize("filt", [True, False])
def test_slicer_oracle_matches_reference_g5(filt):
    """pad_dimensions / index map / 3-view sample_slice / preprocess (mri_dataset.py:11-143)."""
    from oracle.data_ref import build_dataset
    z = _load("g5_slicer.npz")
    _, scans = g5_scans(z)
    key = "filt" if filt else "all"
    dims, imap, items = build_dataset(scans, filt)
    assert tuple(dims) == tuple(z[f"{key}/image_dims"])
    assert np.array_equal(np.array(imap), z[f"{key}/index_map"])
    assert np.array_equal(np.stack([a for a, _ in items]), z[f"{key}/images"])   # bit-exact
    assert np.array_equal(np.stack([b for _, b in items]), z[f"{key}/masks"])


def test_fusion_restatement_g6():
    """The fusion restatement reproduces G6's Dice (computed with the reference's dice_coeff)."""
    from oracle.data_ref import class_dice, fuse
    z = _load("g6_fusion.npz")
    for tag in ("cube", "box"):
        probs = [torch.from_numpy(z[f"{tag}/probs{v}"]) for v in range(3)]
        vols = fuse(*probs)
        assert torch.equal(vols[3], torch.from_numpy(z[f"{tag}/avg"]))
        truth = torch.from_numpy(z[f"{tag}/truth"])
        d = np.array([[class_dice(v, truth, k) for k in (1, 2)] for v in vols])
        assert np.array_equal(d, z[f"{tag}/dice"])


def test_oracle_accumulation_matches_reference_g7():
    """8 micro-batches x loss/8 (train.py:93-98) on c1: the oracle reproduces the reference's
    accumulated gradient (the target the DP all-reduce must hit)."""
    from oracle.unet_ref import unet_forward, unet_loss, unet_param_keys
    z = _load("g7_dp.npz")
    sd = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("init/")}
    keys = unet_param_keys(sd)
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["t"])
    for i in range(8):
        (unet_loss(unet_forward(work, x[4 * i:4 * i + 4], 2, 1), t[4 * i:4 * i + 4], 1) / 8).backward()
    ref = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("grad/")}
    err, key = grad_err({k: params[k].grad for k in keys}, ref)
    assert err <= 1e-5, (err, key)


@pytest.mark.parametrize("n,micro,acc,world", [(103, 2, 4, 2), (64, 4, 4, 4), (50, 1, 1, 2), (77, 8, 4, 8),
                                               (40, 2, 4, 1), (90, 2, 4, 3)])
def test_dp_micro_batches_partition(n, micro, acc, world):
    """The ranks' micro-batches are disjoint and together are exactly the single process's drop_last
    micro-batches (steps of acc, then the trailing ones); every rank has the same step count."""
    from train import dp_micro_batches
    order = list(np.random.default_rng(0).permutation(n))
    per = [dp_micro_batches(order, micro, acc, world, r) for r in range(world)]
    steps = {len(s) for s, _ in per}
    assert len(steps) == 1
    seen = [i for s, left in per for mb in [m for st in s for m in st] + left for i in mb]
    assert len(seen) == len(set(seen))
    for s, left in per:
        assert all(len(mb) == micro for st in s for mb in st) and all(len(mb) == micro for mb in left)
    used = (n // micro) * micro
    assert sorted(seen) == sorted(order[:used])


def test_gpu_only_dropins_refuse_cpu():
    from dice_loss import dice_coeff
    from pmu_hip.fusion import fuse_views
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        dice_coeff(torch.ones(2, 4), torch.ones(2, 4))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        fuse_views(torch.ones(2, 3, 2, 2), torch.ones(2, 3, 2, 2), torch.ones(2, 3, 2, 2), torch.ones(2, 2, 2))
    from utils.mri_dataset import MRI_Dataset
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        MRI_Dataset("imgs", "labs", 3, files=["a"], loader=lambda p: np.zeros((2, 2, 2)), device="cpu")


def test_padded_shape_matches_pad_dimensions():
    from oracle.data_ref import pad_dimensions
    from utils.mri_dataset import padded_shape
    for shp in [(6, 8, 8), (8, 5, 8), (8, 8, 7), (6, 7, 8), (5, 5, 5), (9, 3, 3)]:
        assert padded_shape(shp) == pad_dimensions(np.zeros(shp)).shape
