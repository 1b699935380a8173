"""ProbUNetTrainer — drop-in for PMU/trainer/probunet_trainer.py:10-92."""
import torch

from model import ProbabilisticUnet
from model.probabilistic_unet.utils import l2_regularisation  # noqa: F401  (same import surface)
from pmu_hip.loss import BCELoss, CrossEntropyLoss
from pmu_hip.metrics import trainer_dice

from .trainer import Trainer, load_checkpoint, masks_to_rgb


class ProbUNetTrainer(Trainer):

    def __init__(self, device, n_channels=1, n_classes=1, load_model=None, latent_dim=6, beta=10, num_filters=None):
        """num_filters (extension, train.py --filters): None = the reference's [64..1024] (:16)."""
        self.device = device
        self.mask_type = torch.float32
        self.name = "probunet"
        filters = [64, 128, 256, 512, 1024] if num_filters is None else list(num_filters)
        self.net = ProbabilisticUnet(input_channels=n_channels, num_classes=n_classes,
                                     num_filters=filters, latent_dim=latent_dim, no_convs_fcomb=4,
                                     beta=beta)
        if load_model is not None:
            load_checkpoint(self.net, load_model, device)
        self.net = self.net.to(device)
        self.criterion = BCELoss() if self.net.n_classes == 1 else CrossEntropyLoss()

    def predict(self, imgs, true_masks, z=None):
        """forward (posterior too when grad is enabled) then a prior sample, or logits at ``z`` (:27-32)."""
        train = torch.is_grad_enabled()
        self.net.forward(imgs, true_masks, training=train)
        return self.net.sample(testing=not train) if z is None else self.net.sample_at(z)

    def loss(self, imgs, true_masks, masks_pred):
        """-elbo (:34-39); masks_pred is not used, as in the reference."""
        return -self.net.elbo(true_masks)

    def eval(self, imgs, true_masks, masks_pred):
        return trainer_dice(masks_pred, true_masks, self.net.n_classes)

    def mask_to_image(self, masks, prediction=False):
        return masks_to_rgb(masks, self.net.n_classes, prediction)
