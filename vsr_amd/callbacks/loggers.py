"""Loggers with the reference's names and interface (src/callbacks/loggers/:
BaseLogger base_logger.py:5-59 and the eight ACDC / DSB15 SISR, SISR-SRFB,
MISR and VSR subclasses), so a config's ``logger: {name, kwargs}`` resolves
unchanged (main.py:79-80).

``write(epoch, train_log, train_batch, train_outputs, valid_log, valid_batch,
valid_outputs)`` records the per-epoch scalars as the reference does
(``add_scalars(key, {'train', 'valid'}, epoch)``, base_logger.py:40-48) and
the HR / SR image pair of the last batch (the subclasses' ``_add_images``:
the first sample of ``hr_img`` / ``hr_imgs[-1]`` next to the output).

TensorBoard is used when it is importable.  It is not in this image (nor is
torchvision's make_grid), so the fallback writer keeps the same records in
``log_dir``: ``scalars.jsonl`` (one {"tag", "epoch", "train", "valid"} per
key and epoch) and ``images/{train,valid}_{epoch:04d}.pt`` (the HR | SR grid,
weights-only loadable).  Observability only: nothing here touches the step.
Data-parallel runs write from rank 0 only.
"""
from __future__ import annotations

import json
from pathlib import Path

import torch
import torch.distributed as dist


def _rank0() -> bool:
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


class _FileWriter:
    """The subset of SummaryWriter the loggers use, as plain files."""

    def __init__(self, log_dir):
        self.log_dir = Path(log_dir)
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self._f = open(self.log_dir / "scalars.jsonl", "a")

    def add_scalars(self, tag, values, step):
        self._f.write(json.dumps({"tag": tag, "epoch": int(step), **{k: float(v) for k, v in values.items()}}) + "\n")
        self._f.flush()

    def add_image(self, tag, img, step=None):
        d = self.log_dir / "images"
        d.mkdir(exist_ok=True)
        torch.save(img.detach().cpu(), d / f"{tag}_{int(step or 0):04d}.pt")

    def close(self):
        self._f.close()


def _writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir)
    except ImportError:
        return _FileWriter(log_dir)


def _grid(img: torch.Tensor) -> torch.Tensor:
    """(N, C, H, W) -> (C, N*H + pad, W) column of per-image min-max normalised
    images with white separators (make_grid(nrow=1, normalize=True,
    scale_each=True, pad_value=1), acdc_vsr_logger.py:22-25)."""
    img = img.detach().float()
    lo = img.amin(dim=(1, 2, 3), keepdim=True)
    hi = img.amax(dim=(1, 2, 3), keepdim=True)
    img = (img - lo) / (hi - lo).clamp_min(1e-5)
    n, c, h, w = img.shape
    out = torch.ones((c, n * (h + 2) + 2, w + 4), device=img.device)
    for i in range(n):
        out[:, 2 + i * (h + 2):2 + i * (h + 2) + h, 2:2 + w] = img[i]
    return out


class BaseLogger:
    """base_logger.py:5-59."""

    def __init__(self, log_dir, net=None, dummy_input=None):
        self.writer = _writer(log_dir) if _rank0() else None

    def write(self, epoch, train_log, train_batch, train_outputs, valid_log, valid_batch, valid_outputs):
        if self.writer is None:
            return
        self._add_scalars(epoch, train_log, valid_log)
        self._add_images(epoch, train_batch, train_outputs, valid_batch, valid_outputs)

    def close(self):
        if self.writer is not None:
            self.writer.close()

    def _add_scalars(self, epoch, train_log, valid_log):
        for key in train_log:
            self.writer.add_scalars(key, {'train': train_log[key], 'valid': valid_log[key]}, epoch)

    def _pair(self, batch, outputs):
        """(HR, SR) images the subclass shows."""
        raise NotImplementedError

    def _add_images(self, epoch, train_batch, train_outputs, valid_batch, valid_outputs):
        for tag, batch, outputs in (('train', train_batch, train_outputs), ('valid', valid_batch, valid_outputs)):
            if batch is None or outputs is None:
                continue
            hr, sr = self._pair(batch, outputs)
            self.writer.add_image(tag, torch.cat([_grid(hr), _grid(sr)], dim=-1), epoch)


class AcdcSISRLogger(BaseLogger):
    """acdc_sisr_logger.py: hr_img | output."""

    def _pair(self, batch, outputs):
        return batch['hr_img'], outputs


class AcdcSISRSRFBLogger(BaseLogger):
    """acdc_sisr_srfb_logger.py: hr_img | the last feedback step's output."""

    def _pair(self, batch, outputs):
        return batch['hr_img'], outputs[-1]


class AcdcMISRLogger(AcdcSISRLogger):
    """acdc_misr_logger.py: hr_img | output."""


class AcdcVSRLogger(BaseLogger):
    """acdc_vsr_logger.py:13-30: the last frame's hr_imgs[-1] | outputs[-1]."""

    def _pair(self, batch, outputs):
        return batch['hr_imgs'][-1], outputs[-1]


class Dsb15SISRLogger(AcdcSISRLogger):
    pass


class Dsb15SISRSRFBLogger(AcdcSISRSRFBLogger):
    pass


class Dsb15MISRLogger(AcdcMISRLogger):
    pass


class Dsb15VSRLogger(AcdcVSRLogger):
    pass
