#!/bin/bash
# Round 4: main-stream reduction grid target (PGDIST_WRED_MAIN_WGS; the stem weight-gradient
# reduction at the end of the MobileNetV2 backward, ResNet-50's main-stream reductions)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4w3 && export TMPDIR=/tmp
O=gpurun_out/r4w3
ab() {
  t=$1; x=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py $x > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do
  ab main2048 "--steps 60 --warmup 10" X=1
  ab main128 "--steps 60 --warmup 10" PGDIST_WRED_MAIN_WGS=128
  ab main512 "--steps 60 --warmup 10" PGDIST_WRED_MAIN_WGS=512
done
for i in 1 2; do
  ab rn2048 "--model resnet50 --steps 20 --warmup 5" X=1
  ab rn512 "--model resnet50 --steps 20 --warmup 5" PGDIST_WRED_MAIN_WGS=512
done
