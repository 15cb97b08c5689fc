#!/bin/bash
# Round 4: pw_tile k step 32 everywhere (PGDIST_TILE_K64=4096: half the operand LDS of the
# 64-wide k steps, more room beside the side-stream weight gradients) vs the default
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k64 && export TMPDIR=/tmp
O=gpurun_out/k64
for i in 1 2 3; do
  for v in 256 4096 512; do
    PGDIST_TILE_K64=$v timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('k64 $v', d['ms_per_step'], d['value'])"
  done
done
