"""U-Net (drop-in for PMU/model/unet/unet_model.py).

Same constructor, attributes, module tree and state_dict keys as the reference
(unet_model.py:9-29; up_blocks stored deepest-first, :29).  ``forward`` runs the whole
encoder/decoder on the MI355X HIP engine in one autograd node (pmu_hip.functions.UNetFunction):
  - returns sigmoid(logits) when n_classes == 1, logits otherwise (:48-49);
  - returns the last DoubleConv activation when apply_last_layer is False (:51-54), without
    evaluating the discarded OutConv (:40) — outc then receives no gradient, as in the reference;
  - the reference's per-call torch.cuda.empty_cache() (:46) is dropped.
"""
import torch.nn as nn

from .unet_parts import DoubleConv, Down, OutConv, Up


class UNet(nn.Module):
    def __init__(self, n_channels, n_classes, num_filters=[64, 128, 256, 512, 1024], bilinear=False,
                 apply_last_layer=True):
        super(UNet, self).__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.bilinear = bilinear
        self.apply_last_layer = apply_last_layer
        self.num_filters = num_filters
        # registration order == reference (down_blocks, up_blocks, inc, outc)
        self.down_blocks = nn.ModuleList()
        self.up_blocks = nn.ModuleList()
        # construction order == reference RNG order (inc, outc, then Down/Up pairs)
        self.inc = DoubleConv(n_channels, self.num_filters[0])
        self.outc = OutConv(self.num_filters[0], n_classes)
        for i in range(len(self.num_filters) - 1):
            self.down_blocks.append(Down(self.num_filters[i], self.num_filters[i + 1]))
            self.up_blocks.append(Up(self.num_filters[i + 1], self.num_filters[i], bilinear))
        self.up_blocks = self.up_blocks[::-1]

    def forward(self, x):
        from pmu_hip.functions import unet_apply
        return unet_apply(self, x)
