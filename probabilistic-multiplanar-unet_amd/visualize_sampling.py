"""Latent-grid sampling — drop-in for PMU/visualize_sampling.py.

The reference sweeps two latent components over mu +- k*sigma and, for every grid point, calls
``trainer.predict(slice, mask, z=z)`` — a full forward of the U-Net and both encoders followed by
``sample_at(z)`` (visualize_sampling.py:11-27).  Here the forward runs once and the whole grid is
decoded by one fused Fcomb pass that reads the features once (``ProbabilisticUnet.sample_at`` with
an (S, L) z, ``latent_grid``).  The figure itself (matplotlib) is optional.

One behavioural difference: with the network in train mode the reference's per-point forwards
each update the BatchNorm running statistics (n^2 updates); the single forward here updates them
once.  The decoded logits are identical (train-mode BN uses the slice's own statistics).
"""
from __future__ import annotations

import torch

from model import ProbabilisticUnet

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def sample_grid(train, slice, true_mask, n_preds, mu, sigma):
    """(rows, cols, K, H, W) logits of the latent sweep of visualize_sample, row = z_0 step."""
    with torch.no_grad():
        train.net.forward(slice, true_mask, training=torch.is_grad_enabled())
        z = ProbabilisticUnet.latent_grid(n_preds, mu, sigma)
        y = train.net.sample_at(z)                       # (S, 1, K, H, W)
    n = int(round(z.shape[0] ** 0.5))
    return y[:, 0].reshape(n, n, *y.shape[2:])


def visualize_sample(train, slice, true_mask, n_preds, mu, sigma):
    """visualize_sampling.py:11-53: the grid of predicted masks (mask_to_image of every sample),
    saved as viz_grid.png / viz_scan.png / viz_label.png when matplotlib is available.
    Returns the grid of mask images [[(1, 3, H, W)] * cols] * rows."""
    grid = sample_grid(train, slice, true_mask, n_preds, mu, sigma)
    predictions = [[train.mask_to_image(grid[i, j][None], prediction=True) for j in range(grid.shape[1])]
                   for i in range(grid.shape[0])]
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        import numpy as np
    except ImportError:   # the figure is optional; the samples are the product
        return predictions
    plt.imsave("viz_scan.png", slice.cpu().numpy().squeeze(), cmap="Greys_r")
    mask_img = train.mask_to_image(true_mask, prediction=False).cpu().numpy().squeeze().transpose(1, 2, 0)
    plt.imsave("viz_label.png", mask_img.astype(np.uint8) * 255)
    rows, cols = len(predictions), len(predictions[0])
    fig, ax = plt.subplots(rows, cols, constrained_layout=True, squeeze=False)
    for i in range(rows):
        for j in range(cols):
            ax[i, j].imshow(predictions[i][j].cpu().numpy().squeeze().transpose(1, 2, 0).astype(np.uint8) * 255)
    plt.setp(ax, xticks=[], yticks=[])
    fig.savefig("viz_grid.png", dpi=150)
    plt.close(fig)
    return predictions


if __name__ == "__main__":
    import argparse
    from torch.utils.data import DataLoader
    from trainer import ProbUNetTrainer
    from utils.mri_dataset import MRI_Dataset
    ap = argparse.ArgumentParser(description="Latent-grid sampling of a trained Probabilistic U-Net")
    ap.add_argument("-f", "--load", required=True)
    ap.add_argument("-d", "--dir", required=True, help="dataset dir with images/ and labels/")
    ap.add_argument("-n", "--n-preds", type=int, default=3)
    a = ap.parse_args()
    trainer = ProbUNetTrainer(device, n_channels=1, n_classes=3, load_model=a.load, latent_dim=6)
    dataset = MRI_Dataset(a.dir + "/images", a.dir + "/labels", trainer.net.n_classes)
    pair = next(iter(DataLoader(dataset, batch_size=1, shuffle=True)))
    img = pair["image"].to(device=device, dtype=torch.float32)
    mask = pair["mask"].to(device=device, dtype=torch.float32)
    with torch.no_grad():
        trainer.net.forward(img, mask)
    mu = trainer.net.prior_latent_space.base_dist.loc.squeeze()
    sigma = trainer.net.prior_latent_space.base_dist.scale.squeeze() * 40.0
    visualize_sample(trainer, img, mask, a.n_preds, mu, sigma)
