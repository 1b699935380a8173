"""Stand-alone application of single U-Net blocks on the HIP engine (used when a reference
block is called directly instead of through UNet.forward)."""


def _unsupported(name):
    raise NotImplementedError(f"{name}: call UNet.forward; stand-alone blocks are not wired to the HIP engine yet")


def double_conv_apply(dc, x, pool=None):
    _unsupported("DoubleConv.forward")


def up_apply(up, x1, x2):
    _unsupported("Up.forward")


def outconv_apply(oc, x):
    _unsupported("OutConv.forward")
