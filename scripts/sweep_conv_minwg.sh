#!/bin/bash
# launch-geometry sweeps of the dense-conv kernels (ResNet-50 step, no side stream)
cd $GRAFT_REPO_ROOT
VAR=${VAR:-PGDIST_CONV_MINWG}
for v in ${VALS:-512 256 160}; do
  env $VAR=$v timeout -k 10 120 python bench.py --model resnet50 --steps 10 --warmup 4 --side-stream 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR $v', d['ms_per_step'])" || exit 1
done
