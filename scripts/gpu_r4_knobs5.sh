#!/bin/bash
# Round 4: depthwise ring-depth knobs re-swept on the tall / round-aware small-map geometry
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kn5 && export TMPDIR=/tmp
O=gpurun_out/kn5
for i in 1 2; do
  for v in "X=1" "PGDIST_DW_FDEPTH_SMALL=6" "PGDIST_DW_FDEPTH_SMALL=8" "PGDIST_DW_DDEPTH_S1=4" "PGDIST_DW_DDEPTH_S1=2"; do
    env $v timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('$v', d['ms_per_step'], d['value'])"
  done
done
