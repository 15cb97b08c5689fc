#!/bin/bash
# ResNet-50 side-stream traffic: gentler split reductions (PGDIST_WRED_WGS) and fewer wgrad splits (PGDIST_WGD_TARGET)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
rn() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rb.json 2> $O/rb.err || { tail -20 $O/rb.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rb.json')); print('rn $t', d['ms_per_step'])"
}
for i in 1 2; do rn default X=1; rn wred192 PGDIST_WRED_WGS=192; rn wred128 PGDIST_WRED_WGS=128; rn wgd512 PGDIST_WGD_TARGET=512; rn wgd256 PGDIST_WGD_TARGET=256; done
