#!/bin/bash
# Round 5: 8 data-parallel ranks sharing ONE MI355X (gloo default group, native P2P communicator
# over IPC-mapped staging; RCCL needs one GPU per rank): the world-8 P2P protocol, bucket-cap
# tuning, per-step BN broadcast and the health fields end to end.  NOT an 8-GPU measurement.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5 && export TMPDIR=/tmp
O=gpurun_out/r5
PGDIST_DIST_BACKEND=gloo PGDIST_COMM=p2p timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 8 --steps 6 --warmup 3 \
  --batch-size 32 > $O/rehearsal8.json 2> $O/rehearsal8.err
rc=$?; tail -3 $O/rehearsal8.err; cat $O/rehearsal8.json; exit $rc
