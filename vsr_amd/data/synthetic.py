"""Synthetic 4-D cine volumes (no datasets can be fetched here).

HR raw = clamp(round(mean + std * z), 0, 255) with z a 5x5-box-smoothed
N(0,1) field rescaled to unit variance; LR raw = r x r average pool of HR raw
(a stand-in for the k-space truncation of acdc_preprocess.py:102-180); both
normalized with the dataset constants as the Normalize transform does
(transforms.py:100-168, configs: means/stds 54.089/48.084 for ACDC).
"""
from __future__ import annotations

import torch
import torch.nn.functional as Fn

from ..utils import DATASET_STATS


def synth_cine(batch: int, frames: int, h: int, w: int, r: int, dataset: str = "acdc", seed: int = 1234,
               device: str | torch.device = "cpu"):
    """Returns normalized (lr, hr) of shapes (B, T, h, w) and (B, T, r*h, r*w)."""
    mean, std = DATASET_STATS[dataset]
    g = torch.Generator().manual_seed(seed)
    z = torch.randn((batch * frames, 1, h * r + 4, w * r + 4), generator=g)
    z = Fn.avg_pool2d(z, 5, stride=1) * 5.0  # box smoothing, unit variance again
    hr_raw = (mean + std * z).round().clamp(0, 255)
    lr_raw = Fn.avg_pool2d(hr_raw, r)
    hr = ((hr_raw - mean) / std).reshape(batch, frames, h * r, w * r)
    lr = ((lr_raw - mean) / std).reshape(batch, frames, h, w)
    return lr.to(device), hr.to(device)


def cyclic_windows(vol: torch.Tensor, n: int, order: str = "middle") -> list[torch.Tensor]:
    """(B, T, H, W) -> list of n frames, each (B*T, 1, H, W): for every target
    frame t the window of n frames with cyclic wrap-around over the cardiac
    cycle (acdc_misr_dataset.py:53-68; 'last' = acdc_vsr_dataset.py:59-76)."""
    b, t, h, w = vol.shape
    start = -((n - 1) // 2) if order == "middle" else -(n - 1)
    idx = (torch.arange(t).view(t, 1) + torch.arange(start, start + n).view(1, n)) % t  # (T, n)
    win = vol[:, idx.to(vol.device)]  # (B, T, n, H, W)
    return [win[:, :, k].reshape(b * t, 1, h, w) for k in range(n)]


class SyntheticCine:
    """Map-style dataset with the reference dict contract over synthetic volumes."""

    def __init__(self, task: str, volumes: int = 4, frames: int = 16, size=(128, 128), upscale_factor: int = 4,
                 num_frames: int = 7, dataset: str = "acdc", seed: int = 1234):
        if task not in ("sisr", "misr", "vsr"):
            raise ValueError(task)
        self.task, self.n = task, num_frames
        self.lr, self.hr = synth_cine(volumes, frames, size[0], size[1], upscale_factor, dataset, seed)
        self.volumes, self.frames = volumes, frames

    def __len__(self):
        return self.volumes * self.frames if self.task != "vsr" else self.volumes

    def __getitem__(self, index):
        if self.task == "vsr":
            return {"lr_imgs": [f.unsqueeze(0) for f in self.lr[index]],
                    "hr_imgs": [f.unsqueeze(0) for f in self.hr[index]], "index": index}
        v, t = divmod(index, self.frames)
        if self.task == "sisr":
            return {"lr_img": self.lr[v, t].unsqueeze(0), "hr_img": self.hr[v, t].unsqueeze(0), "index": index}
        start = t - (self.n - 1) // 2
        ids = [(start + k) % self.frames for k in range(self.n)]
        return {"lr_imgs": [self.lr[v, i].unsqueeze(0) for i in ids], "hr_img": self.hr[v, t].unsqueeze(0),
                "index": index}
