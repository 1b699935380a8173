"""Prediction — drop-in for PMU/predict.py:15-19, plus the volume prediction of eval.py:131-203.

``predict(net, imgs, masks, train=True, prob=False)`` keeps the reference signature (for the
probabilistic net: forward, then one prior sample) and returns the prediction (the reference's
body stops before returning it).

``predict_volume`` runs a network over every slice of every view of one resident scan in batches
(the reference feeds eval.py one slice at a time through a DataLoader) and fuses the three views
with one kernel (pmu_hip.fusion): per-view and averaged Dice, the averaged probability volume and
its argmax label map.
"""
from __future__ import annotations

import torch

from pmu_hip.fusion import fuse_views


def predict(net, imgs, masks, train=True, prob=False):
    if prob:
        net.forward(imgs, masks, training=train)
        return net.sample(testing=(not train))
    return net(imgs)


@torch.no_grad()
def predict_volume(net, dataset, scan, batch_size=32, prob=False, n_samples=5, faithful=True):
    """Predict all slices of ``scan`` along the three views and fuse them.

    ``prob``: net is a ProbabilisticUnet; eval.py averages ``n_samples`` prior samples but, as
    written (:148-154), keeps only the first sample divided by n_samples — ``faithful`` reproduces
    that, otherwise the mean of the samples is used.  Returns fuse_views' dict plus the stacks."""
    from utils.mri_dataset import view_slice_shape
    net.eval()
    sv = dataset.scans[scan]
    C = net.n_classes
    stacks = []
    for v in range(3):
        n = sv.pshape[v]
        ha, hb = view_slice_shape(sv.pshape, v)
        out = torch.empty(n, C, ha, hb, dtype=torch.float32, device=dataset.device)
        for s0 in range(0, n, batch_size):
            keys = [(scan, v, s) for s in range(s0, min(n, s0 + batch_size))]
            b = dataset.get_slices(keys)
            if prob:
                net.forward(b["image"], b["mask"], training=False)
                if faithful:
                    y = net.sample(testing=True) / n_samples
                else:
                    y = net.sample_many(n_samples).mean(0)
            else:
                y = net(b["image"])
            out[s0:s0 + len(keys)] = y
        stacks.append(out)
    truth = dataset.get_slices([(scan, 0, s) for s in range(sv.pshape[0])])["mask"][:, 0]
    res = fuse_views(stacks[0], stacks[1], stacks[2], truth, logits=(C > 1))
    res["stacks"] = stacks
    res["truth"] = truth
    return res
