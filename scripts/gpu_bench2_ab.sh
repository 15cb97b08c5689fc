#!/bin/bash
# 2-rank bench rehearsal on one GPU (gloo) under different env settings: B2_ENVS="A=1,B=2 C=3"
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
port=29540
for e in $B2_ENVS; do
  port=$((port+1))
  env $(echo "$e" | tr ',' ' ') PGDIST_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/b2.json 2> gpurun_out/b2.err || { tail -5 gpurun_out/b2.err; exit 4; }
  echo "$e $(python -c "import json;d=json.loads(open('gpurun_out/b2.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done
