#!/bin/bash
# ResNet-50: fewer splits for the 1x1 weight gradients (PGDIST_WGD_T1) with / without gentler reductions
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
rn() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rb.json 2> $O/rb.err || { tail -20 $O/rb.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rb.json')); print('rn $t', d['ms_per_step'])"
}
for i in 1 2; do rn default X=1; rn t1_256 PGDIST_WGD_T1=256; rn t1_128 PGDIST_WGD_T1=128; rn wgd256 PGDIST_WGD_TARGET=256; rn t1_256_wred192 PGDIST_WGD_T1=256 PGDIST_WRED_WGS=192; done
