"""Metrics on HIP kernels, same names/arguments as src/model/metrics.py.

PSNR (metrics.py:9-36) runs as one fused reduction kernel; ``psnr_denorm``
fuses the trainer's denormalize (utils.py:1-20) into it, which is what the
train step calls every iteration (base_trainer.py:135).
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
