"""Trainers with the reference's interface (src/runner/trainers/*.py), running
the train step on the HIP generators.

Same class names, constructor keywords, hook methods (_run_epoch,
_allocate_data, _get_inputs_targets, _compute_losses, _compute_metrics,
_init_log, _update_log, save, load) and log keys ('Loss', one per loss and
metric class name) as BaseTrainer (base_trainer.py:8-253) and its ACDC/DSB15
SISR, SISR-SRFB, MISR and VSR subclasses.  What changes, and why:

  * No host sync per step.  The reference calls .item() on every loss and
    metric of every batch (base_trainer.py:218-222), which serialises the GPU
    with the host each step.  Here they accumulate into device tensors and
    are read once per epoch (the per-step tqdm postfix is therefore not
    printed).  The log values are the same: batch_size-weighted means, with
    the reference's use of dataloader.batch_size for every batch
    (base_trainer.py:137) kept.
  * Metrics run fused: PSNR / SSIM of denormalized images (utils.py:1-20 then
    metrics.py) are single HIP kernels with the denormalize inside.
  * Data parallel: an optional ``grad_sync`` (vsr_amd.ddp.GradSync) is
    finished between backward and optimizer.step(); BatchNorm statistics are
    synchronised across ranks (vsr_amd.ddp.enable_sync_bn) whenever a process
    group with more than one rank is up; the loaders' DistributedSampler
    (vsr_amd.data.Dataloader) gets set_epoch each epoch; logs are
    all-reduced (sum) across ranks once per epoch; checkpoints are written by
    rank 0 only.
  * Checkpoints keep the reference's schema but store the monitor as plain
    state, so ``load`` uses torch.load(weights_only=True) -- also for
    checkpoints written by the reference, whose pickled Monitor is mapped
    onto vsr_amd.callbacks.Monitor by an allow-list (nothing in the file is
    executed).
  * ReduceLROnPlateau: base_trainer.py:67 tests an undefined ``mode`` (a
    NameError whenever that scheduler is used); it is stepped here with the
    validation loss, which is what the branch evidently intends.

The FRVSR trainers (acdc/dsb15_frvsr_trainer.py) belong to a generator this
build does not provide and are not mirrored.
"""
from __future__ import annotations

import functools
import logging
import random

import numpy as np
import torch
import torch.distributed as dist

from .. import metrics as M
from ..callbacks.monitor import Monitor, safe_globals
from ..ddp import enable_sync_bn
from ..utils import denormalize


def _metric(fn, output, target, dataset):
    """metric_fn(denormalize(output), denormalize(target)) -- fused for PSNR/SSIM."""
    if isinstance(fn, M.PSNR) and output.is_cuda:
        m, per = M.F.psnr(output, target, *M.DATASET_STATS[dataset], fn.max_value, denormalize=True)
        return m if fn.size_average else per
    if isinstance(fn, M.SSIM) and output.is_cuda and output.dim() == 4:
        m, per = M.F.ssim(output, target, *M.DATASET_STATS[dataset], fn.value_range, denormalize=True)
        return m if fn.size_average else per
    return fn(denormalize(output, dataset), denormalize(target, dataset))


class BaseTrainer:
    """base_trainer.py:8-253."""

    dataset = "acdc"

    def __init__(self, device, train_dataloader, valid_dataloader, net, loss_fns, loss_weights, metric_fns,
                 optimizer, lr_scheduler, logger, monitor, num_epochs, grad_sync=None):
        self.device = device
        self.train_dataloader = train_dataloader
        self.valid_dataloader = valid_dataloader
        self.net = net.to(device)
        self.loss_fns = [loss_fn.to(device) for loss_fn in loss_fns]
        self.loss_weights = torch.tensor(loss_weights, dtype=torch.float, device=device)
        self.metric_fns = [metric_fn.to(device) for metric_fn in metric_fns]
        self.optimizer = optimizer
        if isinstance(lr_scheduler, torch.optim.lr_scheduler.CyclicLR):
            raise NotImplementedError('Do not support torch.optim.lr_scheduler.CyclicLR scheduler yet.')
        self.lr_scheduler = lr_scheduler
        self.logger = logger
        self.monitor = monitor
        self.num_epochs = num_epochs
        self.epoch = 1
        self.np_random_seeds = None
        self.grad_sync = grad_sync
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            enable_sync_bn(self.net)
        self._denormalize = functools.partial(denormalize, dataset=self.dataset)

    # ------------------------------------------------------------------
    def train(self):
        if self.np_random_seeds is None:
            self.np_random_seeds = random.sample(range(10000000), k=self.num_epochs)
        while self.epoch <= self.num_epochs:
            np.random.seed(self.np_random_seeds[self.epoch - 1])
            for dl in (self.train_dataloader, self.valid_dataloader):
                if hasattr(dl, "set_epoch"):
                    dl.set_epoch(self.epoch)
            logging.info(f'Epoch {self.epoch}.')
            train_log, train_batch, train_outputs = self._run_epoch('training')
            logging.info(f'Train log: {train_log}.')
            valid_log, valid_batch, valid_outputs = self._run_epoch('validation')
            logging.info(f'Valid log: {valid_log}.')
            if self.lr_scheduler is None:
                pass
            elif isinstance(self.lr_scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                self.lr_scheduler.step(valid_log['Loss'])
            else:
                self.lr_scheduler.step()
            if self.logger is not None:
                self.logger.write(self.epoch, train_log, train_batch, train_outputs,
                                  valid_log, valid_batch, valid_outputs)
            if self.monitor is not None:
                saved_path = self.monitor.is_saved(self.epoch)
                if saved_path:
                    logging.info(f'Save the checkpoint to {saved_path}.')
                    self.save(saved_path)
                saved_path = self.monitor.is_best(valid_log)
                if saved_path:
                    logging.info(f'Save the best checkpoint to {saved_path}.')
                    self.save(saved_path)
                if self.monitor.is_early_stopped():
                    logging.info('Early stopped.')
                    break
            self.epoch += 1
        if self.logger is not None:
            self.logger.close()

    def _frames(self, inputs) -> int:
        """Frames per sample in the log weights (1; T for VSR, acdc_vsr_trainer.py:39,56)."""
        return 1

    def _run_epoch(self, mode):
        if mode == 'training':
            self.net.train()
        else:
            self.net.eval()
        dataloader = self.train_dataloader if mode == 'training' else self.valid_dataloader
        log = self._init_log()
        count = 0
        batch = outputs = None
        for batch in dataloader:
            batch = self._allocate_data(batch)
            inputs, targets = self._get_inputs_targets(batch)
            if mode == 'training':
                outputs = self.net(inputs)
                losses = self._compute_losses(outputs, targets)
                loss = (torch.stack(losses) * self.loss_weights).sum()
                self.optimizer.zero_grad()
                loss.backward()
                if self.grad_sync is not None:
                    self.grad_sync.finish()
                # fp16: skip the update of a step whose gradients overflowed (GradScaler)
                if getattr(self.net, "step_ok", None) is None or self.net.step_ok():
                    self.optimizer.step()
            else:
                with torch.no_grad():
                    outputs = self.net(inputs)
                    losses = self._compute_losses(outputs, targets)
                    loss = (torch.stack(losses) * self.loss_weights).sum()
            with torch.no_grad():
                metrics = self._compute_metrics(outputs, targets)
            batch_size = dataloader.batch_size
            T = self._frames(inputs)
            self._update_log(log, batch_size * T, loss, losses, metrics)
            count += batch_size * T
        return self._finish_log(log, count), batch, outputs

    def _finish_log(self, log, count):
        keys = list(log)
        vals = torch.stack([log[k] if torch.is_tensor(log[k]) else torch.tensor(float(log[k]), device=self.device)
                            for k in keys]).double()
        cnt = torch.tensor([float(count)], dtype=torch.float64, device=vals.device)
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(vals)
            dist.all_reduce(cnt)
        vals = (vals / cnt).tolist()  # the one host sync of the epoch
        return dict(zip(keys, vals))

    def _allocate_data(self, batch):
        if isinstance(batch, dict):
            return dict((key, self._allocate_data(data)) for key, data in batch.items())
        elif isinstance(batch, list):
            return list(self._allocate_data(data) for data in batch)
        elif isinstance(batch, tuple):
            return tuple(self._allocate_data(data) for data in batch)
        elif isinstance(batch, torch.Tensor):
            return batch.to(self.device)
        return batch

    def _get_inputs_targets(self, batch):
        raise NotImplementedError

    def _compute_losses(self, outputs, targets):
        raise NotImplementedError

    def _compute_metrics(self, outputs, targets):
        raise NotImplementedError

    def _init_log(self):
        log = {'Loss': 0}
        for loss_fn in self.loss_fns:
            log[loss_fn.__class__.__name__] = 0
        for metric_fn in self.metric_fns:
            log[metric_fn.__class__.__name__] = 0
        return log

    def _update_log(self, log, weight, loss, losses, metrics):
        """log[k] += value * weight, kept on the device (no .item())."""
        log['Loss'] = log['Loss'] + loss.detach().double() * weight
        for loss_fn, lv in zip(self.loss_fns, losses):
            k = loss_fn.__class__.__name__
            log[k] = log[k] + lv.detach().double() * weight
        for metric_fn, mv in zip(self.metric_fns, metrics):
            k = metric_fn.__class__.__name__
            log[k] = log[k] + mv.detach().double() * weight

    def save(self, path):
        """Same checkpoint schema as base_trainer.py:224-237 (state_dict keys of the
        unwrapped net, so reference and vsr_amd checkpoints interoperate); the
        monitor is stored as its state_dict (plain types).  Rank 0 writes."""
        if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            return
        mon = self.monitor
        torch.save({
            'net': self.net.state_dict(),
            'optimizer': self.optimizer.state_dict(),
            'lr_scheduler': self.lr_scheduler.state_dict() if self.lr_scheduler else None,
            'monitor': mon.state_dict() if hasattr(mon, "state_dict") else mon,
            'epoch': self.epoch,
            'random_state': random.getstate(),
            'np_random_seeds': self.np_random_seeds,
        }, path)

    def load(self, path):
        """base_trainer.py:239-252, with torch.load(weights_only=True)."""
        with torch.serialization.safe_globals(safe_globals()):
            checkpoint = torch.load(path, map_location=self.device, weights_only=True)
        self.net.load_state_dict(checkpoint['net'])
        self.optimizer.load_state_dict(checkpoint['optimizer'])
        if checkpoint['lr_scheduler']:
            self.lr_scheduler.load_state_dict(checkpoint['lr_scheduler'])
        state = checkpoint['monitor']
        if state is not None:
            if self.monitor is None:
                d = state if isinstance(state, dict) else vars(state)
                self.monitor = Monitor(d['checkpoints_dir'], d['mode'], d['target'], d['saved_freq'])
            if hasattr(self.monitor, "load_state_dict"):
                self.monitor.load_state_dict(state)
            else:  # a caller-supplied monitor object: restore its attributes
                d = state if isinstance(state, dict) else vars(state)
                for k, v in d.items():
                    if k != "checkpoints_dir":
                        setattr(self.monitor, k, v)
        self.epoch = checkpoint['epoch'] + 1
        random.setstate(checkpoint['random_state'])
        self.np_random_seeds = checkpoint['np_random_seeds']


# ---------------------------------------------------------------- SISR --
class AcdcSISRTrainer(BaseTrainer):
    """acdc_sisr_trainer.py:8-49."""

    dataset = "acdc"

    def _get_inputs_targets(self, batch):
        return batch['lr_img'], batch['hr_img']

    def _compute_losses(self, output, target):
        return [loss_fn(output, target) for loss_fn in self.loss_fns]

    def _compute_metrics(self, output, target):
        return [_metric(fn, output, target, self.dataset) for fn in self.metric_fns]


class Dsb15SISRTrainer(AcdcSISRTrainer):
    """dsb15_sisr_trainer.py (dataset constants of DSB15)."""

    dataset = "dsb15"


class AcdcSISRSRFBTrainer(AcdcSISRTrainer):
    """acdc_sisr_srfb_trainer.py:6-39: feedback nets return one output per step;
    losses are averaged over the steps, metrics use the last step."""

    def _compute_losses(self, outputs, target):
        return [torch.stack([loss_fn(o, target) for o in outputs]).mean() for loss_fn in self.loss_fns]

    def _compute_metrics(self, outputs, target):
        return [_metric(fn, outputs[-1], target, self.dataset) for fn in self.metric_fns]


class Dsb15SISRSRFBTrainer(AcdcSISRSRFBTrainer):
    dataset = "dsb15"


# ---------------------------------------------------------------- MISR --
class AcdcMISRTrainer(AcdcSISRTrainer):
    """acdc_misr_trainer.py:8-49: a window of frames in, the centre frame out."""

    def _get_inputs_targets(self, batch):
        return batch['lr_imgs'], batch['hr_img']


class Dsb15MISRTrainer(AcdcMISRTrainer):
    dataset = "dsb15"


# ----------------------------------------------------------------- VSR --
class AcdcVSRTrainer(BaseTrainer):
    """acdc_vsr_trainer.py:9-123: per-frame mean of losses and metrics, logs
    weighted by batch_size * T."""

    dataset = "acdc"

    def _frames(self, inputs) -> int:
        return len(inputs)

    def _get_inputs_targets(self, batch):
        return batch['lr_imgs'], batch['hr_imgs']

    def _compute_losses(self, outputs, targets):
        return [torch.stack([loss_fn(o, t) for o, t in zip(outputs, targets)]).mean() for loss_fn in self.loss_fns]

    def _compute_metrics(self, outputs, targets):
        return [torch.stack([_metric(fn, o, t, self.dataset) for o, t in zip(outputs, targets)]).mean()
                for fn in self.metric_fns]


class Dsb15VSRTrainer(AcdcVSRTrainer):
    dataset = "dsb15"
