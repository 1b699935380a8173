from .unet_trainer import UNetTrainer
from .probunet_trainer import ProbUNetTrainer
