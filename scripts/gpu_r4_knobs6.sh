#!/bin/bash
# Round 4: executor scheduling knobs re-swept on the final code (side batching, depthwise
# dgrad + wgrad fusion threshold)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kn6 && export TMPDIR=/tmp
O=gpurun_out/kn6
for i in 1 2; do
  for v in "X=1" "PGDIST_SIDE_BATCH=2" "PGDIST_SIDE_BATCH=4" "PGDIST_DW_FUSE_MIN_H=28"; do
    env $v timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('$v', d['ms_per_step'], d['value'])"
  done
done
