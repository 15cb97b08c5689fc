#!/usr/bin/env python3
"""Training entry point (all three reference modes are presets of one config).

  python train.py --preset serial   # cifar10_serial_mobilenet_224.py: CPU, bs=64, torch backend
  python train.py --preset gpu128   # cifar10_128batch.py: 1 GPU, bs=128, native HIP backend
  mpirun -np 8 python train.py --preset mpi          # cifar10_mpi_mobilenet_224.py (+ launch/*.slurm)
  torchrun --nproc-per-node 8 train.py --preset mpi  # same, torchrun rendezvous

Any TrainConfig field can be overridden, e.g. ``--data synthetic --epochs 2``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import pgdist  # noqa: E402,F401
from pgdist.config import TrainConfig, PRESETS, add_cli_args, config_from_args, preset  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None)
    add_cli_args(ap)
    args = ap.parse_args(argv)
    base = preset(args.preset) if args.preset else TrainConfig()
    cfg = config_from_args(args, base)
    from pgdist.engine.trainer import Trainer
    from pgdist.parallel.bootstrap import cleanup
    try:
        Trainer(cfg).fit()
    finally:
        cleanup()


if __name__ == "__main__":
    main()
