"""Dataset constants and denormalize (src/utils.py:1-20)."""
from __future__ import annotations

import torch

# per-dataset intensity mean/std used by Normalize and denormalize (utils.py:13-16)
DATASET_STATS = {"acdc": (54.089, 48.084), "dsb15": (51.193, 52.671)}


def denormalize(imgs: torch.Tensor, dataset: str) -> torch.Tensor:
    """(x*std + mean).round().clamp(0, 255) — utils.py:1-20 (same ValueError on unknown names)."""
    if dataset not in DATASET_STATS:
        raise ValueError(f"The name of the dataset should be 'acdc' or 'dsb15'. Got {dataset}.")
    mean, std = DATASET_STATS[dataset]
    return (imgs.clone() * std + mean).round().clamp(0, 255)
