#!/bin/bash
# Round 4: ResNet-50 implicit-GEMM tile sweep in the replayed step (same box, 2 reps, ms/step)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
ab() {
  t=$1; shift
  env "$@" timeout -k 10 250 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do
  ab default X=1
  ab f128x128 PGDIST_CONV_TILE_FORCE=128x128
  ab f64x128 PGDIST_CONV_TILE_FORCE=64x128
  ab f128x64 PGDIST_CONV_TILE_FORCE=128x64
  ab f64x64 PGDIST_CONV_TILE_FORCE=64x64
  ab minwg512 PGDIST_CONV_MINWG=512
done
