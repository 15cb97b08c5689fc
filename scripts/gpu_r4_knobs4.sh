#!/bin/bash
# Round 4: side-stream join batching and the block-output fusion threshold re-swept on the final
# schedule (same box, 3 reps, bench ms/step)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4k4 && export TMPDIR=/tmp
O=gpurun_out/r4k4
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do
  ab default X=1
  ab side_batch2 PGDIST_SIDE_BATCH=2
  ab side_batch4 PGDIST_SIDE_BATCH=4
  ab side_batch5 PGDIST_SIDE_BATCH=5
  ab fuse_hw49 PGDIST_FUSE_BLOCK_OUT_HW=49
done
