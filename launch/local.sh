#!/bin/bash
# Single-node launcher: N processes (one per GPU) with torchrun's rendezvous on 127.0.0.1.
#   launch/local.sh 8 --preset mpi --data synthetic --epochs 1
set -euo pipefail
N=${1:-1}; shift || true
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$N" -le 1 ]; then exec python train.py "$@"; fi
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
  --master-port "${MASTER_PORT:-29511}" train.py "$@"
