"""Checkpoint policy with the reference's interface (src/callbacks/monitor.py:4-63):
save every `saved_freq` epochs, keep the best by `target` in `mode`, stop
after `early_stop` epochs without improvement (0 = never).

Checkpoints store the monitor as plain state (``state_dict()``), so they load
with ``torch.load(..., weights_only=True)``.  Checkpoints written by the
reference hold a pickled ``src.callbacks.monitor.Monitor``; ``safe_globals()``
names this class (and pathlib's paths) for the weights-only unpickler under
that name, so those load without executing anything from the file either.
"""
from __future__ import annotations

import math
import pathlib


class Monitor:
    def __init__(self, checkpoints_dir, mode, target, saved_freq, early_stop=0):
        self.checkpoints_dir = pathlib.Path(checkpoints_dir)
        self.mode = mode
        self.target = target
        self.saved_freq = saved_freq
        self.early_stop = early_stop if early_stop else math.inf
        self.best = math.inf if mode == "min" else -math.inf
        self.not_improved_count = 0
        self.checkpoints_dir.mkdir(parents=True, exist_ok=True)

    def is_saved(self, epoch):
        """Path of the periodic checkpoint of `epoch`, or None."""
        return self.checkpoints_dir / f"model_{epoch}.pth" if epoch % self.saved_freq == 0 else None

    def is_best(self, valid_log):
        """Path of the best checkpoint when valid_log[target] improved, else None."""
        score = valid_log[self.target]
        better = score > self.best if self.mode == "max" else (score < self.best if self.mode == "min" else False)
        if better:
            self.best = score
            self.not_improved_count = 0
            return self.checkpoints_dir / "model_best.pth"
        self.not_improved_count += 1
        return None

    def is_early_stopped(self):
        return self.not_improved_count == self.early_stop

    # -- checkpoint state (plain types only) --------------------------------
    _KEYS = ("mode", "target", "saved_freq", "early_stop", "best", "not_improved_count")

    def state_dict(self) -> dict:
        return {"checkpoints_dir": str(self.checkpoints_dir), **{k: getattr(self, k) for k in self._KEYS}}

    def load_state_dict(self, state) -> None:
        """From a state_dict() or from the attributes of an unpickled reference Monitor."""
        if not isinstance(state, dict):
            state = dict(vars(state))
        for k in self._KEYS:
            if k in state:
                setattr(self, k, state[k])


def safe_globals() -> list:
    """Allow-list for torch.load(weights_only=True) of reference checkpoints."""
    return [(Monitor, "src.callbacks.monitor.Monitor"), pathlib.PosixPath, pathlib.WindowsPath, pathlib.Path]
