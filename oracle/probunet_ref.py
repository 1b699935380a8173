"""CPU oracle: functional restatement of the reference Probabilistic U-Net (rows a9-a12).

TEST INFRASTRUCTURE ONLY (same rules as oracle/unet_ref.py): imported only by tests/,
__graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg.  Written from scratch on torch
CPU functional ops over a state_dict with the reference's key names
(PMU/ = /root/reference/Probabilistic-Multiplanar-Unet/, PU = PMU/model/probabilistic_unet/).

Randomness is injected: posterior/prior samples are mu + sigma * eps with caller-given eps,
which is exactly what Normal.rsample computes (so gradients flow through mu and sigma).
Pinned by tests/golden/g3_probunet*.npz, produced by importing the reference itself.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .unet_ref import _bn, unet_forward


def encoder_forward(sd, pre, x, n_levels, training=True, convs_per_block=2):
    """Encoder.forward (PU/probabilistic_unet.py:26-53): block i = [AvgPool2d(2,2,0,ceil) if i>0]
    + convs_per_block x (Conv3x3 pad 1 -> BatchNorm2d -> ReLU).  Sequential indices: the pool,
    when present, takes one slot; each conv/bn/relu triple three."""
    idx = 0
    for i in range(n_levels):
        if i > 0:
            x = F.avg_pool2d(x, kernel_size=2, stride=2, padding=0, ceil_mode=True)
            idx += 1
        for _ in range(convs_per_block):
            x = F.conv2d(x, sd[f"{pre}layers.{idx}.weight"], sd[f"{pre}layers.{idx}.bias"], padding=1)
            x = F.relu(_bn(x, sd, f"{pre}layers.{idx + 1}.", training))
            idx += 3
    return x


def gaussian_forward(sd, pre, x, n_levels, latent_dim, segm=None, training=True):
    """AxisAlignedConvGaussian.forward (PU/probabilistic_unet.py:82-114) -> (mu, log_sigma).
    The distribution is Independent(Normal(mu, exp(log_sigma)), 1)."""
    if segm is not None:
        x = torch.cat((x, segm), dim=1)
    enc = encoder_forward(sd, pre + "encoder.", x, n_levels, training)
    enc = enc.mean(dim=2, keepdim=True).mean(dim=3, keepdim=True)           # :97-98
    mls = F.conv2d(enc, sd[pre + "conv_layer.weight"], sd[pre + "conv_layer.bias"])[:, :, 0, 0]
    return mls[:, :latent_dim], mls[:, latent_dim:]


def fcomb_forward(sd, feat, z, n_convs):
    """Fcomb.forward (PU/probabilistic_unet.py:167-181): z broadcast over H x W (tile == expand),
    cat [features, z] -> (1x1 conv -> ReLU) x max(1, n_convs-1) -> last 1x1 conv."""
    N, _, H, W = feat.shape
    zt = z[:, :, None, None].expand(z.shape[0], z.shape[1], H, W)
    x = torch.cat((feat, zt), dim=1)
    for j in range(max(1, n_convs - 1)):
        x = F.relu(F.conv2d(x, sd[f"fcomb.layers.{2 * j}.weight"], sd[f"fcomb.layers.{2 * j}.bias"]))
    return F.conv2d(x, sd["fcomb.last_layer.weight"], sd["fcomb.last_layer.bias"])


def kl_normal(mu_q, ls_q, mu_p, ls_p):
    """Analytic KL(Independent(Normal) q || p), summed over the latent dim
    (torch.distributions kl_normal_normal + Independent, PU/probabilistic_unet.py:272)."""
    var_ratio = torch.exp(2 * (ls_q - ls_p))
    t1 = ((mu_q - mu_p) / torch.exp(ls_p)).pow(2)
    return (0.5 * (var_ratio + t1 - 1 - torch.log(var_ratio))).sum(-1)


def probunet_forward_loss(sd, x, segm, eps_post, n_levels, latent_dim, n_classes, n_convs_fcomb, beta,
                          training=True):
    """ProbabilisticUnet.forward(training=True) + elbo(segm) (PU/probabilistic_unet.py:215-308) with the
    posterior sample mu_q + sigma_q * eps_post.  Returns a dict of the intermediate quantities and
    ``loss`` = -elbo = sum CE(reconstruction, segm) + beta * mean KL."""
    mu_q, ls_q = gaussian_forward(sd, "posterior.", x, n_levels, latent_dim, segm=segm, training=training)
    mu_p, ls_p = gaussian_forward(sd, "prior.", x, n_levels, latent_dim, training=training)
    # unet.* keys carry a prefix; run the U-Net oracle on a prefix-stripped view that writes
    # running statistics back into sd
    usd = {k[5:]: v for k, v in sd.items() if k.startswith("unet.")}
    feat = unet_forward(usd, x, n_levels, n_classes, apply_last_layer=False, training=training)
    for k, v in usd.items():
        sd["unet." + k] = v
    z_q = mu_q + torch.exp(ls_q) * eps_post
    kl = kl_normal(mu_q, ls_q, mu_p, ls_p).mean()
    rec = fcomb_forward(sd, feat, z_q, n_convs_fcomb)
    target = segm.long().squeeze(1)
    ce = F.cross_entropy(rec, target, reduction="none").sum()
    loss = ce + beta * kl
    return dict(mu_q=mu_q, ls_q=ls_q, mu_p=mu_p, ls_p=ls_p, feat=feat, z_q=z_q, kl=kl, rec=rec, ce=ce,
                loss=loss, elbo=-loss)


def probunet_param_keys(sd):
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                  or k.endswith("num_batches_tracked"))]


def probunet_train_step(sd, x, segm, eps_post, n_levels, latent_dim, n_classes, n_convs_fcomb, beta):
    """One training step's forward+backward on CPU; returns (results, grads) and updates sd's
    running statistics (ProbUNetTrainer.loss, PMU/trainer/probunet_trainer.py:34-39)."""
    keys = probunet_param_keys(sd)
    params = {k: sd[k].detach().clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    res = probunet_forward_loss(work, x, segm, eps_post, n_levels, latent_dim, n_classes, n_convs_fcomb, beta)
    res["loss"].backward()
    grads = {k: params[k].grad.detach().clone() if params[k].grad is not None else torch.zeros_like(params[k])
             for k in keys}
    for k in sd:
        if k not in params:
            sd[k] = work[k]
    return {k: v.detach() for k, v in res.items()}, grads
