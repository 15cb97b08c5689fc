#!/bin/bash
# Round 4: depthwise dgrad+wgrad fusion threshold (more wgrad work on the main stream, no
# side-stream re-read of dy / y / x) -- same box, 2 reps, bench ms/step
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do
  ab default X=1
  ab dwfuse28 PGDIST_DW_FUSE_MIN_H=28
  ab dwfuse14 PGDIST_DW_FUSE_MIN_H=14
  ab dwfuse7 PGDIST_DW_FUSE_MIN_H=7
  ab dwfuse112 PGDIST_DW_FUSE_MIN_H=112
done
