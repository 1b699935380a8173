"""Trainer interface — drop-in for PMU/trainer/trainer.py:1-13."""


class Trainer:
    def predict(self, imgs, masks):
        raise NotImplementedError

    def eval(self, imgs, true_masks, masks_pred):
        raise NotImplementedError

    def loss(self, imgs, true_masks, masks_pred):
        raise NotImplementedError

    def mask_to_image(self, mask, prediction=False):
        raise NotImplementedError


# class colours of mask_to_image (unet_trainer.py:107-109, probunet_trainer.py:70-71)
MASK_COLORS = ((0., 0., 0.), (0., 0., 1.), (0., 1., 0.), (1., 0., 0.))


def masks_to_rgb(masks, n_classes, prediction):
    """mask_to_image of both trainers, vectorised (the reference loops over pixels in Python):
    1 class -> (masks >= 0.5) or masks; else a colour per argmax (prediction) or per label value,
    returned (B, 3, H, W) on the CPU like the reference's torch.zeros((batch, h, w, 3)) buffer."""
    import torch
    if n_classes == 1:
        return (masks >= 0.5).float() if prediction else masks
    colors = torch.tensor(MASK_COLORS)
    idx = torch.argmax(masks, dim=1) if prediction else masks.squeeze(1).long()
    return colors[idx.cpu()].permute(0, 3, 1, 2)


def load_checkpoint(net, load_model, device):
    """load_state_dict(torch.load(load_model, map_location=device), strict=False) with the safe
    loader (weights only: a state_dict is plain tensors)."""
    import torch
    net.load_state_dict(torch.load(load_model, map_location=device, weights_only=True), strict=False)
    from pmu_hip.engine import invalidate_packs
    invalidate_packs()   # (load_state_dict bumps the version counters the pack cache checks; belt and braces)
