"""Config surface of the reference (configs/{train,test}/*.yaml read by
src/main.py): YAML -> attribute dict, every object ``{name, kwargs}`` resolved
by name (main.py:167-178 ``_get_instance``).

``python-box`` (the reference's Box, main.py:18) is not installed here; Box
is the small attribute dict below with the methods main.py calls on it
(``from_yaml``, ``get``, ``update``, ``pop``, ``to_dict`` and attribute
access at any depth).  ``build_train`` / ``build_test`` are the composition
root of main.py:16-156 with the namespaces of this package, so the
reference's YAML files resolve unchanged; the build adds two optional
sections (absent in the reference's files, defaults = the reference's
behaviour on one device):

  precision: 'fp32' | 'bf16' | 'fp16'      generator compute dtype (default fp32)
  ddp: {enabled: bool, backend: 'nccl'}   data parallel over torch.distributed
                                           (RCCL on ROCm) when launched by torchrun

Names resolve in this order (main.py:56-99):
  dataset     vsr_amd.data (+ 'ConcatDataset' of several {name, kwargs}: the
              mixed ACDC + DSB15 set of BASELINE config 5)
  dataloader  vsr_amd.data
  net         vsr_amd.nets
  losses      vsr_amd.losses (HIP kernels: L1Loss, MSELoss, HuberLoss,
              CharbonnierLoss), then torch.nn (main.py:60-65 resolves
              torch.nn first; the HIP losses equal torch's within 1e-6 and
              keep the step on the device)
  metrics     vsr_amd.metrics
  optimizer   torch.optim;  lr_scheduler torch.optim.lr_scheduler
  logger      vsr_amd.callbacks.loggers
  monitor     vsr_amd.callbacks
  trainer     vsr_amd.runner.trainers;  predictor vsr_amd.runner.predictors
"""
from __future__ import annotations

import logging
import random
from pathlib import Path

import torch
import torch.nn as nn
import yaml


class Box(dict):
    """Attribute-access dict (nested dicts and lists of dicts become Boxes)."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        for k, v in dict(*args, **kwargs).items():
            self[k] = v

    @staticmethod
    def _wrap(v):
        if isinstance(v, Box):
            return v
        if isinstance(v, dict):
            return Box(v)
        if isinstance(v, (list, tuple)) and any(isinstance(e, dict) for e in v):
            return type(v)(Box._wrap(e) for e in v)
        return v

    def __setitem__(self, k, v):
        super().__setitem__(k, Box._wrap(v))

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    def update(self, *args, **kwargs):
        for k, v in dict(*args, **kwargs).items():
            self[k] = v

    def to_dict(self):
        def un(v):
            if isinstance(v, dict):
                return {k: un(e) for k, e in v.items()}
            if isinstance(v, (list, tuple)):
                return type(v)(un(e) for e in v)
            return v
        return un(self)

    @classmethod
    def from_yaml(cls, yaml_string=None, filename=None):
        if filename is not None:
            yaml_string = Path(filename).read_text()
        return cls(yaml.safe_load(yaml_string) or {})


def get_instance(module, config, *args):
    """main.py:167-178: ``getattr(module, config.name)(*args, **config.kwargs)``."""
    cls = getattr(module, config.name)
    kwargs = config.get('kwargs')
    return cls(*args, **config.kwargs) if kwargs else cls(*args)


def resolve(namespaces, name):
    """The first namespace that defines `name` (AttributeError naming all of them otherwise)."""
    for ns in namespaces:
        if hasattr(ns, name):
            return ns
    raise AttributeError(f"'{name}' is defined in none of {[getattr(n, '__name__', n) for n in namespaces]}")


def seed_everything(random_seed) -> int:
    """main.py:29-33: Python's random seeded with the config value, torch with
    the second word of its state (2613296012 for 'vsr')."""
    random.seed(random_seed)
    torch_seed = random.getstate()[1][1]
    torch.manual_seed(torch_seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(torch_seed)
    return torch_seed


def _namespaces():
    from . import data, losses, metrics, nets
    from .callbacks import loggers
    from . import callbacks
    from .runner import predictors, trainers
    return dict(data=data, losses=losses, metrics=metrics, nets=nets, loggers=loggers, callbacks=callbacks,
                trainers=trainers, predictors=predictors)


def build_dataset(config, type_):
    """dataset section for one split ('train' / 'valid' / 'test'), main.py:42-45,117-119."""
    ns = _namespaces()
    cfg = Box(config.to_dict())
    if cfg.name == 'ConcatDataset':
        parts = [build_dataset(Box(p), type_) for p in cfg.kwargs.datasets]
        return torch.utils.data.ConcatDataset(parts)
    cfg.kwargs.update(data_dir=Path(cfg.kwargs.data_dir), type=type_)
    return get_instance(ns['data'], cfg)


def _collate(config):
    ns = _namespaces()
    name = config.name if config.name != 'ConcatDataset' else config.kwargs.datasets[0]['name']
    return getattr(getattr(ns['data'], name), 'collate_fn', None)


def build_losses(config):
    """losses: [{name, weight[, kwargs]}] -> (loss_fns, loss_weights), main.py:59-67."""
    ns = _namespaces()
    fns, weights = [], []
    for c in config.losses:
        mod = resolve([ns['losses'], nn], c.name)
        fns.append(get_instance(mod, c))
        weights.append(c.weight)
    return fns, weights


def build_metrics(config):
    ns = _namespaces()
    return [get_instance(ns['metrics'], c) for c in config.metrics]


def build_net(config):
    """net section (main.py:56) with the build's precision key applied."""
    ns = _namespaces()
    net = get_instance(ns['nets'], config.net)
    prec = config.get('precision', 'fp32')
    if prec not in ('fp32', 'bf16', 'fp16'):
        raise ValueError(f"precision must be fp32, bf16 or fp16, got {prec!r}")
    if hasattr(net, 'set_precision'):
        net.set_precision(prec)
    return net


def build_train(config, device=None):
    """main.py:16-108 (training branch) -> the trainer, ready for ``train()``."""
    ns = _namespaces()
    config = Box(config.to_dict()) if isinstance(config, Box) else Box(config)
    saved_dir = Path(config.main.saved_dir)
    saved_dir.mkdir(parents=True, exist_ok=True)
    with open(saved_dir / 'config.yaml', 'w+') as f:
        yaml.dump(config.to_dict(), f, default_flow_style=False)
    seed_everything(config.main.random_seed)
    dev_name = device or config.trainer.kwargs.device
    if 'cuda' in str(dev_name) and not torch.cuda.is_available():
        raise ValueError("The cuda is not available. Please set the device in the trainer section to 'cpu'.")
    device = torch.device(dev_name)
    train_dataset = build_dataset(config.dataset, 'train')
    valid_dataset = build_dataset(config.dataset, 'valid')
    dl = Box(config.dataloader.to_dict())
    train_bs, valid_bs = dl.kwargs.pop('train_batch_size'), dl.kwargs.pop('valid_batch_size')
    dl.kwargs.update(collate_fn=_collate(config.dataset), batch_size=train_bs)
    train_loader = get_instance(ns['data'], dl, train_dataset)
    dl.kwargs.update(batch_size=valid_bs, shard_padding=False)  # no repeated samples in the metrics
    valid_loader = get_instance(ns['data'], dl, valid_dataset)
    net = build_net(config)
    loss_fns, loss_weights = build_losses(config)
    metric_fns = build_metrics(config)
    optimizer = get_instance(torch.optim, config.optimizer, net.parameters())
    lr_scheduler = (get_instance(torch.optim.lr_scheduler, config.lr_scheduler, optimizer)
                    if config.get('lr_scheduler') else None)
    lg = Box(config.logger.to_dict())
    lg.kwargs = lg.get('kwargs') or Box()
    lg.kwargs.update(log_dir=saved_dir / 'log', net=net,
                     dummy_input=torch.randn(tuple(lg.kwargs.get('dummy_input', (1, 1, 8, 8)))))
    logger = get_instance(ns['loggers'], lg)
    mon = Box(config.monitor.to_dict())
    mon.kwargs.update(checkpoints_dir=saved_dir / 'checkpoints')
    monitor = get_instance(ns['callbacks'], mon)
    grad_sync = None
    ddp = config.get('ddp') or {}
    if ddp.get('enabled') and torch.distributed.is_available() and torch.distributed.is_initialized():
        from .ddp import GradSync
        net.to(device)
        grad_sync = GradSync(net, torch.distributed.get_world_size())
        grad_sync.broadcast_params()
    tr = Box(config.trainer.to_dict())
    tr.kwargs.update(device=device, train_dataloader=train_loader, valid_dataloader=valid_loader, net=net,
                     loss_fns=loss_fns, loss_weights=loss_weights, metric_fns=metric_fns, optimizer=optimizer,
                     lr_scheduler=lr_scheduler, logger=logger, monitor=monitor)
    if grad_sync is not None:
        tr.kwargs.update(grad_sync=grad_sync)
    trainer = get_instance(ns['trainers'], tr)
    loaded_path = config.main.get('loaded_path')
    if loaded_path:
        logging.info(f'Load the previous checkpoint from "{loaded_path}".')
        trainer.load(Path(loaded_path))
    return trainer


def build_test(config, device=None):
    """main.py:110-156 (testing branch) -> the predictor (weights loaded unless Bicubic)."""
    ns = _namespaces()
    config = Box(config.to_dict()) if isinstance(config, Box) else Box(config)
    dev_name = device or config.predictor.kwargs.device
    if 'cuda' in str(dev_name) and not torch.cuda.is_available():
        raise ValueError("The cuda is not available. Please set the device in the predictor section to 'cpu'.")
    device = torch.device(dev_name)
    test_dataset = build_dataset(config.dataset, 'test')
    dl = Box(config.dataloader.to_dict())
    dl.kwargs = dl.get('kwargs') or Box()
    # the test set is never sharded: under torchrun every rank would otherwise
    # write the same results.csv / PNGs / GIFs from its own shard, and a
    # sequence could straddle two shards; each rank runs the whole set and
    # only rank 0 exports (BasePredictor.predict)
    dl.kwargs.update(shard_padding=False, distributed=False)
    test_loader = get_instance(ns['data'], dl, test_dataset)
    net = build_net(config)
    loss_fns, loss_weights = build_losses(config)
    metric_fns = build_metrics(config)
    pr = Box(config.predictor.to_dict())
    pr.kwargs.update(device=device, test_dataloader=test_loader, net=net, loss_fns=loss_fns,
                     loss_weights=loss_weights, metric_fns=metric_fns)
    predictor = get_instance(ns['predictors'], pr)
    if config.net.name != 'Bicubic' and config.main.get('loaded_path'):
        predictor.load(Path(config.main.loaded_path))
    return predictor
