#!/bin/bash
# A/B of the side-stream CU mask (PGDIST_SIDE_CUS) on the default bench; 3 runs each, interleaved
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for m in 0 1/4 3/8 1/2 5/8; do
  PGDIST_SIDE_CUS=$m timeout -k 10 120 python bench.py --steps 50 --warmup 10 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 4; }
  echo "cus=$m $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'], d['value'])")"
done
done
