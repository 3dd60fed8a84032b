"""Command line of the reference (src/main.py:159-187): ``python -m vsr_amd.main
config.yaml [--test]`` trains (or, with --test, runs the predictor) from a
config in the reference's schema (see vsr_amd.config).

Data parallel: launched by torchrun (RANK / WORLD_SIZE / LOCAL_RANK set) and
with ``ddp: {enabled: true}`` in the config, each process binds its GPU
(LOCAL_RANK), joins the process group (backend 'nccl' = RCCL on ROCm,
MASTER_ADDR / MASTER_PORT from torchrun) and trains its shard; rank 0 writes
logs and checkpoints.
"""
from __future__ import annotations

import argparse
import logging
import os
from pathlib import Path

import torch
import torch.distributed as dist

from . import config as C


def _parse_args(argv=None):
    parser = argparse.ArgumentParser(description="The script for the training and the testing.")
    parser.add_argument('config_path', type=Path, help='The path of the config file.')
    parser.add_argument('--test', action='store_true',
                        help='Perform the testing if specified; otherwise perform the training.')
    return parser.parse_args(argv)


def _init_distributed(config) -> str | None:
    """Process group for a torchrun launch with ddp enabled; returns the device name."""
    ddp = config.get('ddp') or {}
    if not ddp.get('enabled') or int(os.environ.get('WORLD_SIZE', '1')) <= 1:
        return None
    local = int(os.environ.get('LOCAL_RANK', '0'))
    backend = ddp.get('backend', 'nccl')
    if backend == 'nccl':
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return f'cuda:{local}' if backend == 'nccl' else 'cpu'


def main(argv=None):
    args = _parse_args(argv)
    logging.info(f'Load the config from "{args.config_path}".')
    config = C.Box.from_yaml(filename=args.config_path)
    device = _init_distributed(config)
    try:
        if not args.test:
            trainer = C.build_train(config, device=device)
            logging.info('Start training.')
            trainer.train()
            logging.info('End training.')
        else:
            predictor = C.build_test(config, device=device)
            logging.info('Start testing.')
            predictor.predict()
            logging.info('End testing.')
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    logging.basicConfig(format='%(asctime)s | %(levelname)s | %(message)s', level=logging.INFO,
                        datefmt='%Y-%m-%d %H:%M:%S')
    main()
