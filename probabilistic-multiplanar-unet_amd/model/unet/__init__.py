from .unet_model import UNet
