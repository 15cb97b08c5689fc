#!/bin/bash
# Round 4: fused pointwise backward / LDS-resident pointwise forward grid sizes re-swept on the
# final code (defaults: PGDIST_PWB_WGS 512, PGDIST_PW_WGS 2048)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/grids && export TMPDIR=/tmp
O=gpurun_out/grids
for i in 1 2; do
  for v in "X=1" "PGDIST_PWB_WGS=384" "PGDIST_PWB_WGS=640" "PGDIST_PW_WGS=1536" "PGDIST_PW_WGS=3072"; do
    env $v timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('$v', d['ms_per_step'], d['value'])"
  done
done
