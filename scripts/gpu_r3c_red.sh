#!/bin/bash
# weight-gradient split reduction: 4 rows in flight per thread (in-tree) vs 2 (ab/ built with PGDIST_RED_ROWS4=0),
# and reduction grid targets (PGDIST_WRED_WGS) for ResNet-50 / MobileNetV2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_kernels_gpu.py -k "wgrad or reduce" > $O/red_tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/red_tests.log | head -20; tail -3 $O/red_tests.log; exit 1; }
tail -1 $O/red_tests.log
rn() {
  d=$1; t=$2; shift; shift
  (cd $d && env "$@" timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rb.json 2> $O/rb.err) || { tail -20 $O/rb.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rb.json')); print('rn $t', d['ms_per_step'])"
}
mb() {
  d=$1; t=$2; shift; shift
  (cd $d && env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/mb.json 2> $O/mb.err) || { tail -20 $O/mb.err; exit 1; }
  python -c "import json; d=json.load(open('$O/mb.json')); print('mb $t', d['ms_per_step'])"
}
for i in 1 2; do rn . rows4 X=1; rn ab rows2 X=1; rn . rows4_w1024 PGDIST_WRED_WGS=1024; rn . rows4_w2048 PGDIST_WRED_WGS=2048; done
for i in 1 2; do mb . rows4 X=1; mb ab rows2 X=1; done
