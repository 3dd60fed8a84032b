"""Monitor (callbacks/monitor.py mirror) and the trainer's checkpoint round
trip with torch.load(weights_only=True), including a checkpoint in the
reference's own format (pickled src.callbacks.monitor.Monitor)."""
import math
import pathlib
import random
import sys
import types

import torch
import torch.nn as nn

from vsr_amd.callbacks import Monitor
from vsr_amd.runner import trainers


def test_monitor_policy_as_reference(tmp_path):
    # test/callbacks/test_monitor.py:7-15 of the reference
    m = Monitor(tmp_path / "ckpt", mode="min", target="Loss", saved_freq=2, early_stop=2)
    assert m.is_saved(1) is None
    assert m.is_saved(2) == tmp_path / "ckpt" / "model_2.pth"
    assert not m.is_early_stopped()
    assert m.is_best({"Loss": 1.0}) == tmp_path / "ckpt" / "model_best.pth"
    assert m.is_best({"Loss": 2.0}) is None and not m.is_early_stopped()
    assert m.is_best({"Loss": 1.5}) is None and m.is_early_stopped()
    mx = Monitor(tmp_path / "c2", mode="max", target="PSNR", saved_freq=1)
    assert mx.early_stop == math.inf and mx.best == -math.inf
    assert mx.is_best({"PSNR": 20.0}) is not None and mx.is_best({"PSNR": 19.0}) is None


def _trainer(tmp_path, monitor):
    torch.manual_seed(0)
    net = nn.Conv2d(1, 1, 3, padding=1)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.StepLR(opt, 2)
    return trainers.AcdcSISRTrainer(torch.device("cpu"), [], [], net, [nn.L1Loss()], [1.0], [], opt, sched, None,
                                    monitor, 3)


def test_checkpoint_round_trip_weights_only(tmp_path):
    mon = Monitor(tmp_path / "ckpt", mode="max", target="PSNR", saved_freq=1)
    mon.is_best({"PSNR": 31.5})
    tr = _trainer(tmp_path, mon)
    tr.epoch, tr.np_random_seeds = 2, [1, 2, 3]
    p = tmp_path / "model_2.pth"
    tr.save(p)
    torch.load(p, weights_only=True)  # plain types only
    tr2 = _trainer(tmp_path, Monitor(tmp_path / "ckpt", mode="max", target="PSNR", saved_freq=1))
    tr2.load(p)
    assert tr2.epoch == 3 and tr2.np_random_seeds == [1, 2, 3] and tr2.monitor.best == 31.5
    for a, b in zip(tr.net.parameters(), tr2.net.parameters()):
        assert torch.equal(a, b)


def test_reference_checkpoint_loads_weights_only(tmp_path):
    """A checkpoint as base_trainer.py:224-237 writes it: the monitor object
    itself is pickled under src.callbacks.monitor.Monitor."""
    names = ["src", "src.callbacks", "src.callbacks.monitor"]
    for n in names:
        sys.modules[n] = types.ModuleType(n)
    try:
        RefMonitor = type("Monitor", (), {})
        RefMonitor.__module__ = "src.callbacks.monitor"
        sys.modules["src.callbacks.monitor"].Monitor = RefMonitor
        m = RefMonitor()
        m.__dict__.update(checkpoints_dir=pathlib.Path(tmp_path), mode="min", target="Loss", saved_freq=5,
                          early_stop=math.inf, best=0.25, not_improved_count=2)
        tr = _trainer(tmp_path, None)
        p = tmp_path / "ref.pth"
        torch.save({"net": tr.net.state_dict(), "optimizer": tr.optimizer.state_dict(), "lr_scheduler": None,
                    "monitor": m, "epoch": 7, "random_state": random.getstate(), "np_random_seeds": [4]}, p)
    finally:
        for n in names:
            del sys.modules[n]
    tr2 = _trainer(tmp_path, None)
    tr2.load(p)
    assert isinstance(tr2.monitor, Monitor) and tr2.monitor.best == 0.25 and tr2.monitor.not_improved_count == 2
    assert tr2.epoch == 8
