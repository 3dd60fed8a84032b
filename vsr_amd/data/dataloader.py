"""Dataloader with the reference's interface (src/data/dataloader.py:6-53),
sharded across data-parallel ranks.

Same constructor and the same default ``worker_init_fn`` (numpy reseeded per
worker, dataloader.py:52-53).  New: when torch.distributed is initialised
with more than one rank and no sampler is given, a DistributedSampler shards
the (unchanged) Dataset so that each rank sees a disjoint, equally sized part
of every epoch (padded to a multiple of the world size, or trimmed with
drop_last); ``shuffle`` moves into the sampler, seeded identically on every
rank.  The trainer calls ``set_epoch`` so each epoch draws a new permutation.
``shard_padding=False`` (the validation / test loaders of vsr_amd.config)
gives each rank a contiguous, unpadded range instead: no sample is repeated,
so metrics summed over the ranks (BaseTrainer._finish_log) average exactly
the dataset.
"""
from __future__ import annotations

import numpy as np
import torch.distributed as dist
from torch.utils.data import DataLoader, Sampler
from torch.utils.data.distributed import DistributedSampler


class ShardSampler(Sampler):
    """Rank r of w takes the contiguous indices [r*n//w, (r+1)*n//w): no
    padding, no repeats (ranks may differ in size by one sample)."""

    def __init__(self, dataset, num_replicas=None, rank=None):
        self.n = len(dataset)
        self.w = num_replicas if num_replicas is not None else dist.get_world_size()
        self.r = rank if rank is not None else dist.get_rank()

    def __iter__(self):
        return iter(range(self.r * self.n // self.w, (self.r + 1) * self.n // self.w))

    def __len__(self):
        return (self.r + 1) * self.n // self.w - self.r * self.n // self.w


class Dataloader(DataLoader):
    def __init__(self, dataset, batch_size=1, shuffle=False, sampler=None, batch_sampler=None, num_workers=0,
                 collate_fn=None, pin_memory=False, drop_last=False, timeout=0, worker_init_fn=None,
                 distributed=None, seed=0, shard_padding=True):
        if worker_init_fn is None:
            worker_init_fn = self._default_worker_init_fn
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if distributed and sampler is None and batch_sampler is None:
            if shard_padding:
                sampler = DistributedSampler(dataset, shuffle=shuffle, seed=seed, drop_last=drop_last)
            else:
                sampler = ShardSampler(dataset)
            shuffle = False
        kw = dict(dataset=dataset, batch_size=batch_size, shuffle=shuffle, sampler=sampler,
                  batch_sampler=batch_sampler, num_workers=num_workers, pin_memory=pin_memory,
                  drop_last=drop_last, timeout=timeout, worker_init_fn=worker_init_fn)
        if collate_fn is not None:
            kw["collate_fn"] = collate_fn
        super().__init__(**kw)

    def set_epoch(self, epoch: int) -> None:
        """New shard permutation per epoch (no-op without a DistributedSampler)."""
        if isinstance(self.sampler, DistributedSampler):
            self.sampler.set_epoch(epoch)

    @staticmethod
    def _default_worker_init_fn(worker_id):
        np.random.seed(np.random.get_state()[1][0] + worker_id)
