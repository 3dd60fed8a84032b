"""The trainer mirror (vsr_amd.runner.trainers) against the reference's train
loop semantics (base_trainer.py:99-144, acdc_vsr_trainer.py:16-123): the
epoch log is the dataloader.batch_size(-x-T)-weighted mean of the weighted
loss sum, each loss and each metric on denormalized images, computed here
the reference's way (one .item() per value per batch) with the oracle's
PSNR; runs on the CPU with small torch generators (the trainer is
device-agnostic; its fused-metric path is exercised in tests/test_trainer_gpu.py)."""
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from oracle import cpu_nets
from vsr_amd.data import SyntheticCine
from vsr_amd.runner import trainers


class _PSNR(nn.Module):  # a metric fn the trainer applies to denormalized images
    def forward(self, o, t):
        return cpu_nets.psnr(o, t)


class _SISR(nn.Module):
    def __init__(self):
        super().__init__()
        self.c = nn.Conv2d(1, 4, 3, padding=1)
        self.ps = nn.PixelShuffle(2)

    def forward(self, x):
        return self.ps(self.c(x))


class _VSR(_SISR):
    def forward(self, xs):
        return [super(_VSR, self).forward(x) for x in xs]


def _reference_log(net, loader, loss_fns, weights, metric_fns, vsr, dataset="acdc"):
    log, count = {}, 0
    keys = ["Loss"] + [f.__class__.__name__ for f in loss_fns] + [f.__class__.__name__ for f in metric_fns]
    log = {k: 0.0 for k in keys}
    with torch.no_grad():
        for b in loader:
            if vsr:
                x, y = b["lr_imgs"], b["hr_imgs"]
                out = net(x)
                losses = [torch.stack([fn(o, t) for o, t in zip(out, y)]).mean() for fn in loss_fns]
                mets = [torch.stack([fn(cpu_nets.denormalize(o, dataset), cpu_nets.denormalize(t, dataset))
                                     for o, t in zip(out, y)]).mean() for fn in metric_fns]
                w = loader.batch_size * len(x)
            else:
                x, y = b["lr_img"], b["hr_img"]
                out = net(x)
                losses = [fn(out, y) for fn in loss_fns]
                mets = [fn(cpu_nets.denormalize(out, dataset), cpu_nets.denormalize(y, dataset)) for fn in metric_fns]
                w = loader.batch_size
            loss = (torch.stack(losses) * torch.tensor(weights)).sum()
            log["Loss"] += loss.item() * w
            for k, v in zip(keys[1:], losses + mets):
                log[k] += v.item() * w
            count += w
    return {k: v / count for k, v in log.items()}


def _check(trainer_cls, net, ds, vsr):
    loader = DataLoader(ds, batch_size=3, shuffle=False)  # 8 items -> batches 3, 3, 2 (count uses 3 each)
    loss_fns, weights, metric_fns = [nn.L1Loss(), nn.MSELoss()], [1.0, 0.5], [_PSNR()]
    opt = torch.optim.Adam(net.parameters(), lr=1e-2)
    tr = trainer_cls(device=torch.device("cpu"), train_dataloader=loader, valid_dataloader=loader, net=net,
                     loss_fns=loss_fns, loss_weights=weights, metric_fns=metric_fns, optimizer=opt,
                     lr_scheduler=None, logger=None, monitor=None, num_epochs=1)
    got, _, _ = tr._run_epoch("validation")
    ref = _reference_log(net, loader, loss_fns, weights, metric_fns, vsr)
    assert list(got) == list(ref)
    for k in ref:
        assert abs(got[k] - ref[k]) <= 1e-5 * (1 + abs(ref[k])), (k, got[k], ref[k])
    first = tr._run_epoch("training")[0]["Loss"]
    for _ in range(5):
        last = tr._run_epoch("training")[0]["Loss"]
    assert last < first


def test_sisr_trainer_log_matches_reference_loop():
    torch.manual_seed(0)
    _check(trainers.AcdcSISRTrainer, _SISR(), SyntheticCine("sisr", volumes=2, frames=4, size=(8, 8),
                                                             upscale_factor=2), vsr=False)


def test_vsr_trainer_log_matches_reference_loop():
    torch.manual_seed(0)
    _check(trainers.AcdcVSRTrainer, _VSR(), SyntheticCine("vsr", volumes=8, frames=3, size=(8, 8),
                                                          upscale_factor=2), vsr=True)


def test_trainer_names_match_reference():
    for name in ("AcdcSISRTrainer", "AcdcSISRSRFBTrainer", "AcdcMISRTrainer", "AcdcVSRTrainer",
                 "Dsb15SISRTrainer", "Dsb15SISRSRFBTrainer", "Dsb15MISRTrainer", "Dsb15VSRTrainer"):
        assert issubclass(getattr(trainers, name), trainers.BaseTrainer)
