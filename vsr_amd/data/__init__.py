"""Data side of the step: synthetic cine volumes with the reference Dataset
dict contract (src/data/datasets/*: SISR {'lr_img','hr_img'}, MISR
{'lr_imgs': [T], 'hr_img'}, VSR {'lr_imgs': [T], 'hr_imgs': [T]}) and the
k-space LR synthesis of acdc_preprocess.py (Downscale); the reference's
NIfTI Datasets and transforms, and the GPU batch gather over HBM-resident
volumes (DeviceCineBatcher)."""
from . import nifti, transforms
from .dataloader import Dataloader
from .datasets import (AcdcMISRDataset, AcdcSISRDataset, AcdcVSRDataset, Dsb15MISRDataset, Dsb15SISRDataset,
                       Dsb15VSRDataset)
from .device_batch import DeviceCineBatcher
from .downscale import Downscale, downscale_tensor
from .synthetic import SyntheticCine, cyclic_windows, synth_cine

__all__ = ["Dataloader", "Downscale", "downscale_tensor", "SyntheticCine", "cyclic_windows", "synth_cine", "nifti",
           "transforms", "AcdcSISRDataset", "AcdcMISRDataset", "AcdcVSRDataset", "Dsb15SISRDataset",
           "Dsb15MISRDataset", "Dsb15VSRDataset", "DeviceCineBatcher"]
