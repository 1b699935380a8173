"""CPU oracle of the reference's training driver: train_net (PMU/train.py:27-196) for the U-Net.

TEST INFRASTRUCTURE ONLY (same rules as oracle/unet_ref.py).  A from-scratch restatement on the
functional oracle (unet_ref.py) and the restated slicer (data_ref.py), pinned by
tests/golden/g8_train_net.npz — the reference's own train_net run end to end
(tests/golden/make_golden.py g8).  What it restates:
  * the default-RNG stream: random_split (:42), then per DataLoader iterator a base-seed draw
    (torch's _BaseDataLoaderIter) and, for the shuffled train loader, the RandomSampler's own
    seed + permutation (:47-49);
  * micro-batches of batch_size // acc_steps (acc_steps = 4 if batch_size > 4 else 1, drop_last),
    loss / acc_steps, gradients accumulated, every acc_steps micro-batches clip_grad_value_(0.1)
    + SGD(lr, momentum) (:77-110); trailing micro-batches are run but never stepped;
  * the SummaryWriter stream: Loss/train at optimizer steps, and per validation round one
    'images' / 'masks/true' / 'masks/pred' example, Loss/validation, learning_rate, dice/class_k
    or metrics/dice (:119-178), global_step counting micro-batches and validation batches;
  * ReduceLROnPlateau('max' on the Dice for 1 class, else 'min' on the validation loss) (:66,182).
"""
from __future__ import annotations

import numpy as np
import torch

from .unet_ref import sgd_clip_step, trainer_dice, unet_forward, unet_loss, unet_param_keys


def _loader_draw():
    torch.empty((), dtype=torch.int64).random_()


def _random_sampler(n):
    seed = int(torch.empty((), dtype=torch.int64).random_().item())
    return torch.randperm(n, generator=torch.Generator().manual_seed(seed)).tolist()


def mask_to_image(masks, n_classes, prediction=False):
    """UNetTrainer.mask_to_image (trainer/unet_trainer.py:87-115), 1-class branch and the colour map."""
    if n_classes == 1:
        return (masks >= 0.5).float() if prediction else masks
    colors = torch.tensor([[0., 0., 0.], [0., 0., 1.], [0., 1., 0.], [1., 0., 0.]])
    idx = torch.argmax(masks, dim=1) if prediction else masks.squeeze(1).long()
    return colors[idx].permute(0, 3, 1, 2)


def train_net_ref(sd, items, n_levels, n_classes, epochs, batch_size, lr, lrf, lrp, om, val_percent, seed):
    """items: list of (image (1,H,W), mask (1,H,W)) float32 arrays (MRI_Dataset order).
    Returns (final state_dict, scalars [(tag, value, step)], images [(tag, step, tensor)], order)."""
    torch.manual_seed(seed)
    sd = {k: v.clone() for k, v in sd.items()}
    keys = unet_param_keys(sd)
    n = len(items)
    n_val = int(n * val_percent)
    n_train = n - n_val
    perm = torch.randperm(n).tolist()                  # random_split
    tr_idx, va_idx = perm[:n_train], perm[n_train:]
    acc = 4 if batch_size > 4 else 1
    micro = batch_size // acc
    bufs = {k: torch.zeros_like(sd[k]) for k in keys}
    dummy = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([dummy], lr=lr)               # carries the learning rate for the scheduler
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min" if n_classes > 1 else "max", factor=lrf,
                                                       patience=lrp)
    scalars, images, order = [], [], []
    gs = 0

    def batch(idx):
        order.extend(idx)
        x = torch.from_numpy(np.stack([items[i][0] for i in idx]))
        m = torch.from_numpy(np.stack([items[i][1] for i in idx]))
        return x, (m if n_classes == 1 else m.long())

    for _ in range(epochs):
        _loader_draw()
        ord_ = _random_sampler(n_train)
        mbs = [[tr_idx[j] for j in ord_[i:i + micro]] for i in range(0, n_train - micro + 1, micro)]
        grads = None
        for i, mb in enumerate(mbs):
            x, t = batch(mb)
            params = {k: sd[k].detach().clone().requires_grad_(True) for k in keys}
            work = dict(sd)
            work.update(params)
            loss = unet_loss(unet_forward(work, x, n_levels, n_classes), t, n_classes) / acc
            loss.backward()
            for k in sd:
                if k not in params:
                    sd[k] = work[k]                      # BN running statistics
            g = {k: params[k].grad for k in keys}
            grads = g if grads is None else {k: grads[k] + g[k] for k in keys}
            if (i + 1) % acc == 0:
                scalars.append(("Loss/train", float(loss.detach()), gs))
                cur = {k: sd[k].detach() for k in keys}
                sgd_clip_step(cur, grads, bufs, opt.param_groups[0]["lr"], om, 0.1)
                sd.update(cur)
                grads = None
            gs += 1
        # validation
        _loader_draw()
        vbs = [va_idx[i:i + micro] for i in range(0, n_val - micro + 1, micro)]
        vc = len(vbs)
        dices, dsum, lsum = 0.0, np.zeros(max(0, n_classes - 1)), 0.0
        for mb in vbs:
            x, t = batch(mb)
            with torch.no_grad():
                y = unet_forward(sd, x, n_levels, n_classes, training=False)
                d = np.array(trainer_dice(y, t, n_classes))
                lsum += float(unet_loss(y, t, n_classes))
            if n_classes > 1:
                dsum += d
            else:
                dices += d
            if gs % vc == 0:
                images += [("images", gs, x), ("masks/true", gs, mask_to_image(t, n_classes)),
                           ("masks/pred", gs, mask_to_image(y, n_classes, True))]
            gs += 1
        avg = lsum / vc
        scalars += [("Loss/validation", avg, gs), ("learning_rate", opt.param_groups[0]["lr"], gs)]
        for c in range(n_classes - 1):
            scalars.append((f"dice/class_{c + 1}", dsum[c] / vc, gs))
        if n_classes == 1:
            score = float((dices / vc)[0])
            scalars.append(("metrics/dice", score, gs))
        else:
            score = avg
        sched.step(score)
    return sd, scalars, images, order
