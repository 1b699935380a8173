"""UNetTrainer — drop-in for PMU/trainer/unet_trainer.py:10-129.

Same constructor, attributes (device, name, mask_type, net, criterion) and methods.  The net runs
on the HIP path (model.UNet); the loss is BCELoss / CrossEntropyLoss on HIP kernels (pmu_hip.loss,
row a6; same constructors and reductions as torch's); eval's per-class Dice comes from one fused
argmax+count kernel (pmu_hip.metrics).
"""
import torch

from model import UNet
from pmu_hip.loss import BCELoss, CrossEntropyLoss
from pmu_hip.metrics import trainer_dice

from .trainer import Trainer, load_checkpoint, masks_to_rgb


class UNetTrainer(Trainer):

    def __init__(self, device, n_channels=1, n_classes=1, load_model=None, num_filters=None):
        """num_filters (extension, train.py --filters): the U-Net widths; None = the reference's default."""
        self.device = device
        self.name = "unet"
        self.mask_type = torch.float32 if n_classes == 1 else torch.long
        if num_filters is None:
            self.net = UNet(n_channels=n_channels, n_classes=n_classes)
        else:
            self.net = UNet(n_channels=n_channels, n_classes=n_classes, num_filters=list(num_filters))
        if load_model is not None:
            load_checkpoint(self.net, load_model, device)
        self.net = self.net.to(device)
        self.criterion = BCELoss() if self.net.n_classes == 1 else CrossEntropyLoss()

    def predict(self, imgs, true_masks):
        return self.net(imgs)

    def loss(self, imgs, true_masks, masks_pred):
        if self.net.n_classes > 1:
            return self.criterion(masks_pred, true_masks.squeeze(1))
        return self.criterion(masks_pred, true_masks)

    def eval(self, imgs, true_masks, masks_pred):
        """[dice] for 1 class, else Dice of classes 1..K-1 of the softmax-argmax one-hot (:52-98)."""
        return trainer_dice(masks_pred, true_masks, self.net.n_classes)

    def mask_to_image(self, masks, prediction=False):
        return masks_to_rgb(masks, self.net.n_classes, prediction)
