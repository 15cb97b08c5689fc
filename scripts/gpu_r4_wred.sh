#!/bin/bash
# Round 4: side-stream reduction grid (PGDIST_WRED_WGS) re-A/B, MobileNetV2 and ResNet-50
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4w && export TMPDIR=/tmp
O=gpurun_out/r4w
ab() {
  t=$1; x=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py $x > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3 4; do
  ab default "--steps 60 --warmup 10" X=1
  ab wred128 "--steps 60 --warmup 10" PGDIST_WRED_WGS=128
  ab wred64 "--steps 60 --warmup 10" PGDIST_WRED_WGS=64
done
for i in 1 2; do
  ab rn_default "--model resnet50 --steps 20 --warmup 5" X=1
  ab rn_wred128 "--model resnet50 --steps 20 --warmup 5" PGDIST_WRED_WGS=128
done
