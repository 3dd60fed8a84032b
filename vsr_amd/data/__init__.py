"""Data side of the step: synthetic cine volumes with the reference Dataset
dict contract (src/data/datasets/*: SISR {'lr_img','hr_img'}, MISR
{'lr_imgs': [T], 'hr_img'}, VSR {'lr_imgs': [T], 'hr_imgs': [T]})."""
from .dataloader import Dataloader
from .synthetic import SyntheticCine, cyclic_windows, synth_cine

__all__ = ["Dataloader", "SyntheticCine", "cyclic_windows", "synth_cine"]
