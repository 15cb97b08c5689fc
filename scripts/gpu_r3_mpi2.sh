#!/bin/bash
# 2-rank mpi preset on one GPU (gloo process group + native P2P gradient buckets), per-step
# BN broadcast, replica check at the end
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/e2e && export TMPDIR=/tmp
O=gpurun_out/e2e
PGDIST_COMM=p2p timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 train.py --preset mpi --data synthetic --epochs 2 --dist-backend gloo --max-steps-per-epoch 80 \
  --bn-sync broadcast --save-path $O/best_mpi.pth > $O/mpi_2rank_gloo_p2p_broadcast.log 2>&1 || { tail -20 $O/mpi_2rank_gloo_p2p_broadcast.log; exit 1; }
grep -v amdgpu.ids $O/mpi_2rank_gloo_p2p_broadcast.log | tail -12
