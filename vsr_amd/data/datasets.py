"""The reference's Datasets (src/data/datasets/*.py) over NIfTI volumes, with
the same constructors, directory layout, windowing and sample dicts, so the
configs' ``dataset.name`` / ``kwargs`` resolve here unchanged:

  {data_dir}/{type}/HR/<patient>/*2d+1d*.nii.gz           (H, W, 1, T) HR
  {data_dir}/{type}/LR/X{r}/<patient>/*2d+1d*.nii.gz      (h, w, 1, T) LR

(acdc_preprocess.py:55-85 writes them; the SISR datasets read *2d*.nii.gz
(H, W, 1) slices).  NIfTI is read by vsr_amd.data.nifti (nibabel restated).

Samples (CPU, exactly the reference's):
  SISR  {'lr_img': (C,h,w), 'hr_img': (C,H,W), 'index'}      acdc_sisr_dataset.py:40-52
  MISR  {'lr_imgs': [n x (C,h,w)], 'hr_img', 'index'}        acdc_misr_dataset.py:44-81
  VSR   {'lr_imgs': [n], 'hr_imgs': [n], 'index'} (train) /
        the whole sequence (valid / test)                      acdc_vsr_dataset.py:37-90
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
from torch.utils.data import Dataset

from . import nifti
from .transforms import compose


class BaseDataset(Dataset):
    """base_dataset.py:5-15."""

    def __init__(self, data_dir, type):
        super().__init__()
        self.data_dir = Path(data_dir)
        self.type = type


def _window(t: int, n: int, T: int, order: str):
    """(start, end) of the n-frame window around target t (acdc_vsr_dataset.py:59-64)."""
    if order == "last":
        return t - n + 1, t + 1
    return t - (n - 1) // 2, t + ((n - 1) - (n - 1) // 2) + 1


def _take(imgs: np.ndarray, start: int, end: int) -> np.ndarray:
    """Cyclic frame range over the last axis (acdc_vsr_dataset.py:65-75)."""
    T = imgs.shape[-1]
    if start < 0:
        return np.concatenate((imgs[..., start:], imgs[..., :end]), axis=-1)
    if end > T:
        return np.concatenate((imgs[..., start:], imgs[..., :end % T]), axis=-1)
    return imgs[..., start:end]


class _Seq(BaseDataset):
    default_order = "last"

    def __init__(self, downscale_factor, transforms, augments=None, num_frames=5, temporal_order=None, **kwargs):
        super().__init__(**kwargs)
        if downscale_factor not in [2, 3, 4]:
            raise ValueError(f"The downscale factor should be 2, 3, 4. Got {downscale_factor}.")
        self.downscale_factor = downscale_factor
        self.transforms = compose(transforms)
        self.augments = compose(augments)
        self.num_frames = num_frames
        temporal_order = temporal_order or self.default_order
        if temporal_order not in ["last", "middle"]:
            raise ValueError(f"The temporal order should be 'last' or 'middle'. Got {temporal_order}.")
        self.temporal_order = temporal_order
        self.lr_paths = sorted((self.data_dir / self.type / "LR" / f"X{downscale_factor}").glob("**/*2d+1d*.nii.gz"))
        self.hr_paths = sorted((self.data_dir / self.type / "HR").glob("**/*2d+1d*.nii.gz"))

    def _frames(self, index):
        raise NotImplementedError

    def _sample_imgs(self, lr_imgs, hr_imgs):
        imgs = [lr_imgs[..., t] for t in range(lr_imgs.shape[-1])] + \
               [hr_imgs[..., t] for t in range(hr_imgs.shape[-1])]  # list of (H, W, C)
        if self.type == "train":
            imgs = self.augments(*imgs)
        imgs = self.transforms(*imgs)
        imgs = [img.permute(2, 0, 1).contiguous() for img in imgs]
        return imgs[:len(imgs) // 2], imgs[len(imgs) // 2:]


class AcdcSISRDataset(BaseDataset):
    """acdc_sisr_dataset.py:8-52 (2-D slices)."""

    def __init__(self, downscale_factor, transforms, augments=None, **kwargs):
        super().__init__(**kwargs)
        if downscale_factor not in [2, 3, 4]:
            raise ValueError(f"The downscale factor should be 2, 3, 4. Got {downscale_factor}.")
        self.downscale_factor = downscale_factor
        self.transforms = compose(transforms)
        self.augments = compose(augments)
        lr = sorted((self.data_dir / self.type / "LR" / f"X{downscale_factor}").glob("**/*2d*.nii.gz"))
        hr = sorted((self.data_dir / self.type / "HR").glob("**/*2d*.nii.gz"))
        self.data = list(zip(lr, hr))

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        lr_path, hr_path = self.data[index]
        lr_img = nifti.load(lr_path).get_data()
        hr_img = nifti.load(hr_path).get_data()
        if self.type == "train":
            lr_img, hr_img = self.augments(lr_img, hr_img)
        lr_img = self.transforms(lr_img).permute(2, 0, 1).contiguous()
        hr_img = self.transforms(hr_img).permute(2, 0, 1).contiguous()
        return {"lr_img": lr_img, "hr_img": hr_img, "index": index}


class AcdcMISRDataset(_Seq):
    """acdc_misr_dataset.py:8-81: an n-frame window (default 'middle') per
    target frame, target = the window's centre HR frame."""

    default_order = "middle"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.data = []
        for lp, hp in zip(self.lr_paths, self.hr_paths):
            T = nifti.load(lp).header.get_data_shape()[-1]
            self.data.extend([(lp, hp, t) for t in range(T)])

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        lp, hp, t = self.data[index]
        lr_imgs, hr_imgs = nifti.load(lp).get_data(), nifti.load(hp).get_data()
        s, e = _window(t, self.num_frames, lr_imgs.shape[-1], self.temporal_order)
        lr, hr = self._sample_imgs(_take(lr_imgs, s, e), _take(hr_imgs, s, e))
        c = self.num_frames // 2 if self.num_frames % 2 == 1 else self.num_frames // 2 - 1
        return {"lr_imgs": lr, "hr_img": hr[c], "index": index}


class AcdcVSRDataset(_Seq):
    """acdc_vsr_dataset.py:7-90: train = an n-frame window (default 'last')
    per target frame; valid / test = the whole sequence."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.type == "train":
            self.data = []
            for lp, hp in zip(self.lr_paths, self.hr_paths):
                T = nifti.load(lp).header.get_data_shape()[-1]
                self.data.extend([(lp, hp, t) for t in range(T)])
        else:
            self.data = list(zip(self.lr_paths, self.hr_paths))

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        if self.type == "train":
            lp, hp, t = self.data[index]
        else:
            lp, hp = self.data[index]
        lr_imgs, hr_imgs = nifti.load(lp).get_data(), nifti.load(hp).get_data()
        if self.type == "train":
            s, e = _window(t, self.num_frames, lr_imgs.shape[-1], self.temporal_order)
            lr_imgs, hr_imgs = _take(lr_imgs, s, e), _take(hr_imgs, s, e)
        lr, hr = self._sample_imgs(lr_imgs, hr_imgs)
        return {"lr_imgs": lr, "hr_imgs": hr, "index": index}


# dsb15_*_dataset.py: the same code over the DSB15 directory tree
class Dsb15SISRDataset(AcdcSISRDataset):
    pass


class Dsb15MISRDataset(AcdcMISRDataset):
    pass


class Dsb15VSRDataset(AcdcVSRDataset):
    pass
