"""The reference's data transforms (src/data/transforms.py), for the datasets
of vsr_amd.data.datasets, plus their batched device counterpart.

CPU transforms (numpy in, same names, kwargs, random draws and errors as the
reference, so a config's ``dataset.transforms`` / ``augments`` list builds the
same pipeline): ``compose``, ``Compose``, ``ToTensor``, ``Normalize``,
``RandomCrop``, ``RandomCropPatch``, ``RandomHorizontalFlip``,
``RandomVerticalFlip``.  RandomElasticDeformation needs SimpleITK (absent
here) and is not provided.

Device path: ``plan_augments`` replays the same draws (Python ``random``, in
the reference's order) for a batch and folds each sample's crop / flip chain
into one affine index map, which ``vsrk_gather_windows`` (include/vsrk_data.h)
applies to HBM-resident volumes in one launch (vsr_amd.data.device_batch).
"""
from __future__ import annotations

import random

import numpy as np
import torch


def compose(transforms=None):
    """transforms.py:10-28: a list of {name, kwargs} (Box or dict) -> Compose;
    None -> Compose([ToTensor()])."""
    if transforms is None:
        return Compose([ToTensor()])
    out = []
    for t in transforms:
        name = t["name"] if isinstance(t, dict) else t.name
        kwargs = t.get("kwargs") if isinstance(t, dict) or hasattr(t, "get") else None
        cls = globals()[name]
        out.append(cls(**kwargs) if kwargs else cls())
    return Compose(out)


class BaseTransform:
    def __call__(self, *imgs, **kwargs):
        raise NotImplementedError

    def __repr__(self):
        return self.__class__.__name__


class Compose(BaseTransform):
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, *imgs, **kwargs):
        for t in self.transforms:
            imgs = t(*imgs, **kwargs)
        return imgs[0] if len(imgs) == 1 else imgs

    def __repr__(self):
        return self.__class__.__name__ + "(" + "".join(f"\n    {t}" for t in self.transforms) + "\n)"


def _check_np(imgs):
    if not all(isinstance(img, np.ndarray) for img in imgs):
        raise TypeError("All of the images should be numpy.ndarray.")


def _check_ndim(imgs):
    if not all(img.ndim == 3 for img in imgs) and not all(img.ndim == 4 for img in imgs):
        raise ValueError("All of the images' dimensions should be 3 (2D images) or 4 (3D images).")


class ToTensor(BaseTransform):
    """transforms.py:74-97."""

    def __call__(self, *imgs, dtypes=None, **kwargs):
        _check_np(imgs)
        if dtypes:
            if not all(isinstance(d, torch.dtype) for d in dtypes):
                raise TypeError("All of the dtypes should be torch.dtype.")
            if len(dtypes) != len(imgs):
                raise ValueError("The number of the dtypes should be the same as the images.")
            return tuple(torch.from_numpy(np.ascontiguousarray(i)).to(d) for i, d in zip(imgs, dtypes))
        return tuple(torch.from_numpy(np.ascontiguousarray(i)).float() for i in imgs)


class Normalize(BaseTransform):
    """transforms.py:100-168: per-channel (x - mean) / (std + 1e-10), or the
    image's own statistics when no means / stds are given."""

    def __init__(self, means=None, stds=None):
        if (means is None) != (stds is None):
            raise ValueError("Both the means and the standard deviations should have values or None.")
        if means is not None and len(means) != len(stds):
            raise ValueError("The number of the means should be the same as the standard deviations.")
        self.means, self.stds = means, stds

    def __call__(self, *imgs, normalize_tags=None, **kwargs):
        _check_np(imgs)
        if normalize_tags:
            if len(normalize_tags) != len(imgs):
                raise ValueError("The number of the tags should be the same as the images.")
            if not all(t in [True, False] for t in normalize_tags):
                raise ValueError("All of the tags should be either True or False.")
        else:
            normalize_tags = [None] * len(imgs)
        out = []
        for img, tag in zip(imgs, normalize_tags):
            if tag is None or tag is True:
                if self.means is None:
                    axis = tuple(range(img.ndim - 1))
                    img = self._normalize(img, img.mean(axis=axis), img.std(axis=axis))
                else:
                    img = self._normalize(img, self.means, self.stds)
            out.append(img)
        return tuple(out)

    @staticmethod
    def _normalize(img, means, stds):
        img = img.copy()
        for c, mean, std in zip(range(img.shape[-1]), means, stds):
            img[..., c] = (img[..., c] - mean) / (std + 1e-10)
        return img


def _coords(img, size):
    """transforms.py:207-227 (RandomCrop._get_coordinates): the draws."""
    if any(i - j < 0 for i, j in zip(img.shape, size)):
        raise ValueError(f"The image ({img.shape}) is smaller than the cropped size ({size}). "
                         "Please use a smaller cropped size.")
    if img.ndim == 3:
        h, w = img.shape[:-1]
        ht, wt = size
        h0, w0 = random.randint(0, h - ht), random.randint(0, w - wt)
        return h0, h0 + ht, w0, w0 + wt
    h, w, d = img.shape[:-1]
    ht, wt, dt = size
    h0, w0, d0 = random.randint(0, h - ht), random.randint(0, w - wt), random.randint(0, d - dt)
    return h0, h0 + ht, w0, w0 + wt, d0, d0 + dt


class RandomCrop(BaseTransform):
    """transforms.py:171-227: one random window for every image."""

    def __init__(self, size):
        self.size = size

    def __call__(self, *imgs, **kwargs):
        _check_np(imgs)
        _check_ndim(imgs)
        ndim = imgs[0].ndim
        if ndim - 1 != len(self.size):
            raise ValueError(f"The dimensions of the cropped size should be the same as the image ({ndim - 1}). "
                             f"Got {len(self.size)}")
        c = _coords(imgs[0], self.size)
        if ndim == 3:
            return tuple(img[c[0]:c[1], c[2]:c[3]] for img in imgs)
        return tuple(img[c[0]:c[1], c[2]:c[3], c[4]:c[5]] for img in imgs)


class RandomCropPatch(BaseTransform):
    """transforms.py:373-450: LR images (first half) at a random window, HR
    images (second half) at the corresponding window scaled by `ratio`."""

    def __init__(self, size, ratio):
        self.size = size
        self.ratio = ratio

    def __call__(self, *imgs, **kwargs):
        _check_np(imgs)
        _check_ndim(imgs)
        ndim = imgs[0].ndim
        if ndim - 1 != len(self.size):
            raise ValueError(f"The dimensions of the cropped size should be the same as the image ({ndim - 1}). "
                             f"Got {len(self.size)}")
        if len(imgs) % 2 == 1:
            raise ValueError("The number of the LR images should be the same as the HR images")
        lr, hr = imgs[:len(imgs) // 2], imgs[len(imgs) // 2:]
        if not all(j // i == self.ratio for a, b in zip(lr, hr) for i, j in zip(a.shape[:-1], b.shape[:-1])):
            raise ValueError(f"The ratio between the HR images and the LR images should be {self.ratio}.")
        c = _coords(lr[0], self.size)
        r = self.ratio
        if ndim == 3:
            h0, hn, w0, wn = c
            return tuple([x[h0:hn, w0:wn] for x in lr] + [x[h0 * r:hn * r, w0 * r:wn * r] for x in hr])
        h0, hn, w0, wn, d0, dn = c
        return tuple([x[h0:hn, w0:wn, d0:dn] for x in lr] + [x[h0 * r:hn * r, w0 * r:wn * r, d0:dn] for x in hr])


class RandomHorizontalFlip(BaseTransform):
    """transforms.py:321-345: np.flip(img, 1) with probability prob."""

    def __init__(self, prob=0.5):
        self.prob = max(0, min(prob, 1))

    def __call__(self, *imgs, **kwargs):
        _check_np(imgs)
        _check_ndim(imgs)
        if random.random() < self.prob:
            imgs = tuple(np.flip(img, 1) for img in imgs)
        return imgs


class RandomVerticalFlip(BaseTransform):
    """transforms.py:348-370: np.flip(img, 0) with probability prob."""

    def __init__(self, prob=0.5):
        self.prob = max(0, min(prob, 1))

    def __call__(self, *imgs, **kwargs):
        _check_np(imgs)
        _check_ndim(imgs)
        if random.random() < self.prob:
            imgs = tuple(np.flip(img, 0) for img in imgs)
        return imgs


# ------------------------------------------------------------- device maps --
class IndexMap:
    """src (y, x) = (y0 + dy * y, x0 + dx * x) for an output of (h, w): the
    fold of a crop / flip chain over 2-D images."""

    def __init__(self, h: int, w: int):
        self.y0, self.dy, self.x0, self.dx, self.h, self.w = 0, 1, 0, 1, h, w

    def crop(self, h0: int, w0: int, ht: int, wt: int) -> None:
        self.y0 += self.dy * h0
        self.x0 += self.dx * w0
        self.h, self.w = ht, wt

    def hflip(self) -> None:  # np.flip(img, 1)
        self.x0 += self.dx * (self.w - 1)
        self.dx = -self.dx

    def vflip(self) -> None:  # np.flip(img, 0)
        self.y0 += self.dy * (self.h - 1)
        self.dy = -self.dy


def plan_augments(augments, lr_hw, hr_hw=None):
    """Replay `augments` (a Compose / list of the transforms above, or None)
    for ONE sample of 2-D LR images of size lr_hw (and HR images hr_hw): the
    same `random` draws in the same order as applying them to the numpy
    images, folded into (lr_map, hr_map).  Only RandomCrop (single-size),
    RandomCropPatch and the two flips have device maps; Normalize / ToTensor
    are value transforms the caller applies to the whole volume once."""
    ts = augments.transforms if isinstance(augments, Compose) else (augments or [])
    lm = IndexMap(*lr_hw)
    hm = IndexMap(*hr_hw) if hr_hw is not None else None
    r = hr_hw[0] // lr_hw[0] if hr_hw is not None else 1
    for t in ts:
        if isinstance(t, RandomCropPatch):
            if len(t.size) != 2:
                raise NotImplementedError("device maps cover 2-D images")
            if hm is not None and t.ratio != r:
                raise ValueError(f"The ratio between the HR images and the LR images should be {t.ratio}.")
            h0, hn, w0, wn = _coords(np.empty((lm.h, lm.w, 1), np.uint8), t.size)
            lm.crop(h0, w0, hn - h0, wn - w0)
            if hm is not None:
                hm.crop(h0 * r, w0 * r, (hn - h0) * r, (wn - w0) * r)
        elif isinstance(t, RandomCrop):
            if hm is not None:
                raise NotImplementedError("RandomCrop over LR and HR images of different sizes")
            h0, hn, w0, wn = _coords(np.empty((lm.h, lm.w, 1), np.uint8), t.size)
            lm.crop(h0, w0, hn - h0, wn - w0)
        elif isinstance(t, RandomHorizontalFlip):
            if random.random() < t.prob:
                lm.hflip()
                if hm is not None:
                    hm.hflip()
        elif isinstance(t, RandomVerticalFlip):
            if random.random() < t.prob:
                lm.vflip()
                if hm is not None:
                    hm.vflip()
        elif isinstance(t, (Normalize, ToTensor)):
            continue
        else:
            raise NotImplementedError(f"no device map for {t}")
    return lm, hm
