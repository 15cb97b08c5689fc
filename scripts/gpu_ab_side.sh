#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() { env "${@:2}" timeout -k 10 120 python bench.py --steps 50 --warmup 10 $1 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; return 0; }
  echo "$* -> $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'])")"; }
for rep in 1 2; do
run "--side-stream 0" X=0
run "--side-stream 1" X=0
run "--side-stream 1" PGDIST_SIDE_BATCH=1
run "--side-stream 1" PGDIST_SIDE_BATCH=2
run "--side-stream 1" PGDIST_SIDE_BATCH=4
run "--side-stream 1" PGDIST_SIDE_BATCH=6
run "--side-stream 1" PGDIST_DW_FUSE_MIN_H=112
run "--side-stream 1" PGDIST_DW_FUSE_MIN_H=200
done
