"""Data side of the step: synthetic cine volumes with the reference Dataset
dict contract (src/data/datasets/*: SISR {'lr_img','hr_img'}, MISR
{'lr_imgs': [T], 'hr_img'}, VSR {'lr_imgs': [T], 'hr_imgs': [T]}) and the
k-space LR synthesis of acdc_preprocess.py (Downscale)."""
from .dataloader import Dataloader
from .downscale import Downscale, downscale_tensor
from .synthetic import SyntheticCine, cyclic_windows, synth_cine

__all__ = ["Dataloader", "Downscale", "downscale_tensor", "SyntheticCine", "cyclic_windows", "synth_cine"]
