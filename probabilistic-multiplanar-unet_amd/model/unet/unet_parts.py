"""Parameter containers of the U-Net blocks (drop-in for PMU/model/unet/unet_parts.py).

The blocks keep the reference's module tree — ``double_conv = [Conv2d, BatchNorm2d, ReLU,
Conv2d, BatchNorm2d, ReLU]`` (unet_parts.py:14-21), ``maxpool_conv = [MaxPool2d, DoubleConv]``
(:31-34), ``up`` / ``conv`` (:46-53), ``OutConv.conv`` (:73) — so that state_dict keys and the
default-initialisation RNG order are identical to the reference.  Their arithmetic never
runs in PyTorch: ``UNet.forward`` hands the whole stack to the HIP engine
(``pmu_hip.engine``), which fuses BN+ReLU, pooling, padding and concatenation into the conv
kernels.  Calling a block on its own runs that block on the same engine, as one autograd node
with a materialised output (``pmu_hip.blocks``).
"""
import torch.nn as nn


def conv_bn_relu(cin, cout):
    """The three modules of one conv3x3 -> BatchNorm2d(batch stats) -> ReLU stage."""
    return [nn.Conv2d(cin, cout, kernel_size=3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]


class DoubleConv(nn.Module):
    """(conv3x3 => BatchNorm2d => ReLU) * 2   (reference: unet_parts.py:9-24)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        stages = conv_bn_relu(in_channels, out_channels) + conv_bn_relu(out_channels, out_channels)
        self.double_conv = nn.Sequential(*stages)

    def forward(self, x):
        from pmu_hip.blocks import double_conv_apply
        return double_conv_apply(self, x)


class Down(nn.Module):
    """MaxPool2d(2) then DoubleConv   (reference: unet_parts.py:27-38)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    def forward(self, x):
        from pmu_hip.blocks import down_apply
        return down_apply(self, x)


class Up(nn.Module):
    """ConvTranspose2d(k2, s2) -> pad to the skip -> cat([skip, up]) -> DoubleConv
    (reference: unet_parts.py:41-67).  ``bilinear=True`` is rejected: the reference
    constructor passes three arguments to the two-argument DoubleConv (unet_parts.py:50)
    and cannot be built either."""

    def __init__(self, in_channels, out_channels, bilinear=True):
        super().__init__()
        if bilinear:
            raise TypeError("Up(bilinear=True) is not constructible in the reference "
                            "(DoubleConv takes 2 channel arguments, unet_parts.py:50)")
        self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x1, x2):
        from pmu_hip.blocks import up_apply
        return up_apply(self, x1, x2)


class OutConv(nn.Module):
    """1x1 conv head   (reference: unet_parts.py:70-76)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)

    def forward(self, x):
        from pmu_hip.blocks import outconv_apply
        return outconv_apply(self, x)
