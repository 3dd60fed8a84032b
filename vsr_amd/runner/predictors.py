"""Test-time loop mirror of src/runner/predictors (resolved by name, main.py:110-156).

BasePredictor (base_predictor.py:6-136) and the ACDC / DSB15 SISR, MISR and
VSR predictors (acdc_{sisr,misr,vsr}_predictor.py, dsb15_*): batch size 1,
the network in eval mode, per-frame losses and metrics on the HIP kernels
(PSNR / SSIM fused with denormalize, Cardiac* by patient name), the same
log keys, and -- with ``exported=True`` -- the results CSV (one row per
frame: name, metrics, losses), a PNG per SR frame and a GIF per sequence.

Export names follow the reference exactly: the patient / sequence / frame
ids are parsed from the dataset's file names (SISR ``<patient>_2d_<slice>_<frame>``,
MISR / VSR ``<patient>_2d+1d_<sequence>`` with the frame index t of the
sample), images are ``imgs/<patient>/<slice>_<frame>.png`` and one GIF per
sequence ``videos/<patient>/<sequence>.gif`` (SISR / MISR collect the frames
of a sequence and write its GIF when the sequence id changes).

Differences: images are written with PIL (the reference's scipy.misc.imsave
was removed from SciPy and imageio is not a dependency here); checkpoints
load with ``weights_only=True`` (a reference checkpoint's pickled Monitor
resolves through the same allow-list as the trainer's); the SISR / MISR
predictors also write the GIF of the LAST sequence, which the reference's
loop never flushes (acdc_sisr_predictor.py:72-79 only writes on a change),
and start a new GIF when the patient changes even if the sequence id does
not (the reference keys on the sequence id alone, so two consecutive
single-slice patients would share one GIF).
"""
from __future__ import annotations

import csv
import logging
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from .. import metrics as M
from ..callbacks.monitor import safe_globals
from ..utils import denormalize
from .trainers import _metric


class BasePredictor:
    """base_predictor.py:6-136."""

    dataset_name = "acdc"

    def __init__(self, device, test_dataloader, net, loss_fns, loss_weights, metric_fns, saved_dir=None,
                 exported=False):
        self.device = device
        self.test_dataloader = test_dataloader
        self.net = net.to(device)
        self.loss_fns = [fn.to(device) for fn in loss_fns]
        self.loss_weights = torch.tensor(loss_weights, dtype=torch.float, device=device)
        self.metric_fns = [fn.to(device) for fn in metric_fns]
        if getattr(test_dataloader, "batch_size", 1) != 1:
            raise ValueError(f"The testing batch size should be 1. Got {test_dataloader.batch_size}.")
        self.exported = exported
        self.saved_dir = Path(saved_dir) if exported else None

    # -- reference hooks ------------------------------------------------------
    def _allocate_data(self, batch):
        if isinstance(batch, dict):
            return {k: self._allocate_data(v) for k, v in batch.items()}
        if isinstance(batch, list):
            return [self._allocate_data(v) for v in batch]
        if isinstance(batch, tuple):
            return tuple(self._allocate_data(v) for v in batch)
        if isinstance(batch, torch.Tensor):
            return batch.to(self.device)
        return batch

    def _init_log(self):
        log = {"Loss": 0.0}
        for fn in self.loss_fns:
            log[fn.__class__.__name__] = 0.0
        for fn in self.metric_fns:
            log[fn.__class__.__name__] = 0.0
        return log

    def load(self, path):
        """base_predictor.py:130-136 (net state only), without unpickling code."""
        with torch.serialization.safe_globals(safe_globals()):
            ckpt = torch.load(path, map_location=self.device, weights_only=True)
        self.net.load_state_dict(ckpt["net"])

    # -- per-frame pieces (shared by the SISR / MISR / VSR predictors) ----------
    def _frame_losses(self, outputs, targets):
        """(T, #loss_fns) -- acdc_vsr_predictor.py:118-130."""
        return torch.stack([torch.stack([fn(o, t) for o, t in zip(outputs, targets)]) for fn in self.loss_fns],
                           dim=1)

    def _frame_metrics(self, outputs, targets, name):
        """(T, #metric_fns) on denormalized frames -- acdc_vsr_predictor.py:132-151."""
        rows = []
        for fn in self.metric_fns:
            vals = []
            for o, t in zip(outputs, targets):
                if "Cardiac" in fn.__class__.__name__:
                    vals.append(fn(denormalize(o, self.dataset_name), denormalize(t, self.dataset_name), name))
                else:
                    vals.append(_metric(fn, o, t, self.dataset_name))
            rows.append(torch.stack([v.reshape(()) for v in vals]))
        return torch.stack(rows, dim=1)

    def _sample_name(self, index):
        """(filename, patient, sequence id, frame id or None) of sample `index`
        from the dataset's file names (acdc_vsr_predictor.py:55-58,
        acdc_misr_predictor.py:56-59,68, acdc_sisr_predictor.py:56-58)."""
        data = getattr(self.test_dataloader.dataset, "data", None)
        if data is None:  # a dataset without file names (synthetic)
            return f"sample_2d+1d_sequence{int(index):02d}", "sample", f"sequence{int(index):02d}", "frame01"
        entry = data[int(index)]
        filename = Path(entry[0]).parts[-1].split(".")[0]
        parts = filename.split("_")
        fid = f"frame{int(entry[2]) + 1:0>2d}" if len(entry) > 2 else "frame01"  # MISR: the window's target frame
        return filename, parts[0], parts[2], fid

    def _to_uint8(self, x):
        return denormalize(x, self.dataset_name).squeeze().detach().cpu().numpy().astype(np.uint8)

    @staticmethod
    def _save_png(path, img):
        from PIL import Image
        Image.fromarray(img).save(path)

    @staticmethod
    def _dump_video(path, imgs):
        """acdc_vsr_predictor.py:172-180: the SR frames as one GIF."""
        from PIL import Image
        frames = [Image.fromarray(i) for i in imgs]
        frames[0].save(path, save_all=True, append_images=frames[1:], loop=0)

    # -- export (results rows, PNG per SR frame, GIF per sequence) ---------------
    def _dirs(self, patient):
        vdir, idir = self.saved_dir / "videos" / patient, self.saved_dir / "imgs" / patient
        vdir.mkdir(parents=True, exist_ok=True)
        idir.mkdir(parents=True, exist_ok=True)
        return vdir, idir

    def _flush_video(self, state):
        """GIF of the collected frames of the current sequence (SISR / MISR)."""
        if state["sr_imgs"]:
            vdir, _ = self._dirs(state["patient"])
            self._dump_video(vdir / f"{self._video_name(state['sid'])}.gif", state["sr_imgs"])
            state["sr_imgs"] = []

    def _video_name(self, sid):
        return sid

    @staticmethod
    def _row_name(filename, fid):
        return filename.replace("2d+1d", "2d").replace("sequence", "slice") + f"_{fid}"

    def _export(self, state, results, filename, patient, sid, fid, outs, metrics, losses):
        """One sample holding frame `fid` of sequence `sid` (SISR / MISR: a
        frame; acdc_misr_predictor.py:66-91, acdc_sisr_predictor.py:66-90)."""
        row = torch.cat([metrics, losses], dim=1)[0].cpu().tolist()
        results.append([self._row_name(filename, fid), *row])
        if (patient, sid) != (state["patient"], state["sid"]):
            self._flush_video(state)
        img = self._to_uint8(outs[0])
        state["sr_imgs"].append(img)
        state["sid"], state["patient"] = sid, patient
        _, idir = self._dirs(patient)
        self._save_png(idir / (sid.replace("sequence", "slice") + f"_{fid}.png"), img)

    # -- the loop ---------------------------------------------------------------
    def _get_inputs_targets(self, batch):
        raise NotImplementedError

    def _frames_of(self, outputs, targets):
        """Per-frame lists (T entries)."""
        raise NotImplementedError

    def predict(self):
        self.net.eval()
        # data-parallel launch (torchrun): the test loader is unsharded
        # (vsr_amd.config.build_test) and only rank 0 writes the exports
        exported = self.exported and not (dist.is_available() and dist.is_initialized() and dist.get_rank() != 0)
        header = (["name"] + [fn.__class__.__name__ for fn in self.metric_fns] +
                  [fn.__class__.__name__ for fn in self.loss_fns])
        results = [header]
        state = {"sr_imgs": [], "sid": None, "patient": None}
        log = self._init_log()
        count = 0
        for batch in self.test_dataloader:
            batch = self._allocate_data(batch)
            inputs, targets, index = self._get_inputs_targets(batch)
            with torch.no_grad():
                filename, patient, sid, fid = self._sample_name(index)
                outputs = self.net(inputs)
                outs, tgts = self._frames_of(outputs, targets)
                losses = self._frame_losses(outs, tgts)                  # (T, L)
                loss = (losses.mean(dim=0) * self.loss_weights).sum()
                metrics = self._frame_metrics(outs, tgts, patient)      # (T, M)
            T = len(outs)
            if exported:
                self._export(state, results, filename, patient, sid, fid, outs, metrics, losses)
            # acdc_vsr_predictor.py:160-170: frame-weighted
            log["Loss"] += loss.item() * T
            for fn, v in zip(self.loss_fns, losses.mean(dim=0)):
                log[fn.__class__.__name__] += v.item() * T
            for fn, v in zip(self.metric_fns, metrics.mean(dim=0)):
                log[fn.__class__.__name__] += v.item() * T
            count += T
        if exported:
            self._flush_video(state)
            self.saved_dir.mkdir(parents=True, exist_ok=True)
            with open(self.saved_dir / "results.csv", "w", newline="") as fh:
                csv.writer(fh).writerows(results)
        for k in log:
            log[k] /= max(count, 1)
        logging.info(f"Test log: {log}.")
        return log


class AcdcVSRPredictor(BasePredictor):
    """acdc_vsr_predictor.py:15-180: list of T LR frames -> T SR frames."""

    def _get_inputs_targets(self, batch):
        return batch["lr_imgs"], batch["hr_imgs"], batch["index"]

    def _frames_of(self, outputs, targets):
        return list(outputs), list(targets)

    def _export(self, state, results, filename, patient, sid, fid, outs, metrics, losses):
        """A whole sequence (acdc_vsr_predictor.py:66-96): one row, one PNG per
        frame, the sequence's GIF."""
        stem = filename.replace("2d+1d", "2d").replace("sequence", "slice")
        for t, row in enumerate(torch.cat([metrics, losses], dim=1).cpu().tolist()):
            results.append([stem + f"_frame{t + 1:0>2d}", *row])
        imgs = [self._to_uint8(o) for o in outs]
        vdir, idir = self._dirs(patient)
        self._dump_video(vdir / f"{sid}.gif", imgs)
        for t, img in enumerate(imgs):
            self._save_png(idir / (sid.replace("sequence", "slice") + f"_frame{t + 1:0>2d}.png"), img)


class Dsb15VSRPredictor(AcdcVSRPredictor):
    dataset_name = "dsb15"


class AcdcMISRPredictor(BasePredictor):
    """acdc_misr_predictor.py: T LR frames -> the centre SR frame."""

    @staticmethod
    def _row_name(filename, fid):
        return filename.replace("2d+1d", "2d").replace("sequence", "slice") + f"_{fid}"

    def _get_inputs_targets(self, batch):
        return batch["lr_imgs"], batch["hr_img"], batch["index"]

    def _frames_of(self, output, target):
        return [output], [target]


class Dsb15MISRPredictor(AcdcMISRPredictor):
    dataset_name = "dsb15"


class AcdcSISRPredictor(BasePredictor):
    """acdc_sisr_predictor.py: one LR slice -> one SR slice."""

    def _sample_name(self, index):
        """<patient>_2d_<slice>_<frame> (acdc_sisr_predictor.py:56-58)."""
        filename, patient, sid, _ = super()._sample_name(index)
        parts = filename.split("_")
        return filename, patient, sid, parts[3] if len(parts) > 3 else "frame01"

    @staticmethod
    def _row_name(filename, fid):
        return filename

    def _video_name(self, sid):
        return sid.replace("slice", "sequence")

    def _get_inputs_targets(self, batch):
        return batch["lr_img"], batch["hr_img"], batch["index"]

    def _frames_of(self, output, target):
        return [output], [target]


class Dsb15SISRPredictor(AcdcSISRPredictor):
    dataset_name = "dsb15"


class AcdcSISRSRFBPredictor(AcdcSISRPredictor):
    """acdc_sisr_srfb_predictor.py: feedback nets return every step; losses
    are averaged over the steps (:94-108), metrics score the last (:110-128)."""

    def _frames_of(self, outputs, target):
        self._steps = (list(outputs), target)
        return [outputs[-1]], [target]

    def _frame_losses(self, outs, tgts):
        steps, target = self._steps
        return torch.stack([torch.stack([fn(o, target) for o in steps]).mean() for fn in self.loss_fns]).view(1, -1)


class Dsb15SISRSRFBPredictor(AcdcSISRSRFBPredictor):
    dataset_name = "dsb15"


__all__ = ["BasePredictor", "AcdcVSRPredictor", "Dsb15VSRPredictor", "AcdcMISRPredictor", "Dsb15MISRPredictor",
           "AcdcSISRPredictor", "Dsb15SISRPredictor", "AcdcSISRSRFBPredictor", "Dsb15SISRSRFBPredictor", "M"]
