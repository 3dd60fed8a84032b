"""Metrics on HIP kernels, same names/arguments as src/model/metrics.py.

PSNR (metrics.py:9-36) and SSIM (metrics.py:39-113) each run as one fused
kernel plus a fixed-order final reduction; ``psnr_denorm`` / ``ssim_denorm``
fuse the trainer's denormalize (utils.py:1-20) into them, which is what the
train step calls every iteration (base_trainer.py:135).  CardiacPSNR /
CardiacSSIM (metrics.py:116-165) crop the cardiac bounding box (a view) and
reuse them.  SSIM(dim=3) filters depth first (vsrk_ssim3d).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as F
from .utils import DATASET_STATS


def psnr_denorm(output: torch.Tensor, target: torch.Tensor, dataset: str, max_value: float = 255.0,
                size_average: bool = True) -> torch.Tensor:
    """PSNR(denormalize(output), denormalize(target)) in one kernel."""
    mean, std = DATASET_STATS[dataset]
    m, per = F.psnr(output, target, mean, std, max_value, denormalize=True)
    return m if size_average else per


class PSNR(nn.Module):
    """metrics.py:9-36 — 10*log10(max^2 / (mse + 1e-10)) per sample, then mean."""

    def __init__(self, size_average=True, max_value=255):
        super().__init__()
        self.size_average = size_average
        self.max_value = max_value

    def forward(self, output, target):
        m, per = F.psnr(output, target, max_value=self.max_value, denormalize=False)
        return m if self.size_average else per


def ssim_denorm(output: torch.Tensor, target: torch.Tensor, dataset: str, size_average: bool = True) -> torch.Tensor:
    """SSIM(denormalize(output), denormalize(target)) in one kernel (2-D window)."""
    mean, std = DATASET_STATS[dataset]
    m, per = F.ssim(output, target, mean, std, 255.0, denormalize=True)
    return m if size_average else per


class SSIM(nn.Module):
    """metrics.py:39-113: Gaussian 11^dim window (sigma 1.5), valid filtering; dim 2 or 3."""

    def __init__(self, dim=2, channels=1, size_average=True, value_range=255):
        super().__init__()
        if dim not in (2, 3):
            raise ValueError(f"Only dim=2, 3 are supported. Received dim={dim}.")
        self.dim = dim
        self.channels = channels
        self.size_average = size_average
        self.value_range = value_range
        self.c1 = (0.01 * value_range) ** 2
        self.c2 = (0.03 * value_range) ** 2

    def forward(self, output, target):
        if output.dim() != self.dim + 2:
            raise ValueError(f"SSIM(dim={self.dim}) expects (N, C, *) with {self.dim} spatial dims, "
                             f"got {tuple(output.shape)}")
        m, per = F.ssim(output, target, value_range=self.value_range)
        return m if self.size_average else per


def _load_coordinates(path):
    """{patient name: (h0, hn, w0, wn)}.  The reference reads a pickle
    (metrics.py:123-125) written by its preprocessing; that format is read here
    with an unpickler that resolves no globals (only dict / tuple / list / str
    / int / float containers can be built, nothing in the file is executed).
    A JSON map {name: [h0, hn, w0, wn]} is accepted too."""
    import json
    import pickle

    class _DataOnly(pickle.Unpickler):
        def find_class(self, module, name):
            raise pickle.UnpicklingError(f"coordinates file references {module}.{name}: only plain data is read")

    with open(path, "rb") as fh:
        head = fh.read(1)
        fh.seek(0)
        if head in (b"{", b" ", b"\n"):
            data = json.loads(fh.read().decode())
        else:
            data = _DataOnly(fh).load()
    return {str(k): tuple(int(x) for x in v) for k, v in data.items()}


class CardiacPSNR(nn.Module):
    """metrics.py:116-139: PSNR inside the patient's cardiac bounding box."""

    def __init__(self, coordinates_path, **kwargs):
        super().__init__()
        self.psnr = PSNR(**kwargs)
        self.coordinates = _load_coordinates(coordinates_path)

    def forward(self, output, target, name):
        h0, hn, w0, wn = self.coordinates[name]
        return self.psnr(output[..., h0:hn, w0:wn], target[..., h0:hn, w0:wn])


class CardiacSSIM(nn.Module):
    """metrics.py:142-165: SSIM inside the patient's cardiac bounding box."""

    def __init__(self, coordinates_path, **kwargs):
        super().__init__()
        self.ssim = SSIM(**kwargs)
        self.coordinates = _load_coordinates(coordinates_path)

    def forward(self, output, target, name):
        h0, hn, w0, wn = self.coordinates[name]
        return self.ssim(output[..., h0:hn, w0:wn], target[..., h0:hn, w0:wn])
