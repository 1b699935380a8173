"""Weight initialisers of the Probabilistic U-Net (drop-in for PMU/model/probabilistic_unet/utils.py:7-36).

They must consume the CPU RNG exactly like the reference (one ``normal_`` of shape
``size + (4,)`` per truncated bias, then the weight initialiser) so that a seeded construction
gives bit-identical weights; tests/test_probunet_cpu.py checks this against the reference's G3
initial state_dict.
"""
import torch
import torch.nn as nn


def truncated_normal_(tensor, mean=0.0, std=1.0):
    """Fill ``tensor`` with N(0,1) truncated to (-2, 2), then scale/shift (utils.py:7-13).

    Four candidate draws per element; the first one inside (-2, 2) is kept (index 0 when none is,
    as argmax of an all-False row)."""
    cand = tensor.new_empty(tuple(tensor.shape) + (4,)).normal_()
    inside = (cand > -2) & (cand < 2)
    first = inside.max(-1, keepdim=True)[1]
    with torch.no_grad():
        tensor.copy_(cand.gather(-1, first).squeeze(-1))
        tensor.mul_(std).add_(mean)
    return tensor


def _is_conv(m):
    return type(m) in (nn.Conv2d, nn.ConvTranspose2d)


def init_weights(m):
    """He-normal (fan_in, relu) weight + truncated-normal(0, 1e-3) bias (utils.py:15-20)."""
    if _is_conv(m):
        nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
        truncated_normal_(m.bias, mean=0.0, std=0.001)


def init_weights_orthogonal_normal(m):
    """Orthogonal weight + truncated-normal(0, 1e-3) bias (utils.py:22-26)."""
    if _is_conv(m):
        nn.init.orthogonal_(m.weight)
        truncated_normal_(m.bias, mean=0.0, std=0.001)


def l2_regularisation(m):
    """Sum of the L2 norms of all parameters of ``m`` (utils.py:28-36)."""
    total = None
    for w in m.parameters():
        total = w.norm(2) if total is None else total + w.norm(2)
    return total
