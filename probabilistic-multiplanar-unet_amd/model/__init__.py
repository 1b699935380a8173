"""Drop-in model package (reference: PMU/model/__init__.py): ``from model import UNet, ProbabilisticUnet``."""
from .unet.unet_model import UNet
from .probabilistic_unet import ProbabilisticUnet
