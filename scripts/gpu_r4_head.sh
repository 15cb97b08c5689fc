#!/bin/bash
# Round 4: head CE fused into the head backward, classifier weight gradient on the side stream:
# numerics, executor tests, bench A/B against ab/base (previous commit)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/head && export TMPDIR=/tmp
O=gpurun_out/head
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_bn_fused_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ab() {
  t=$1; b=$2
  timeout -k 10 200 python -u $b --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do ab base ab/base/bench.py; ab new bench.py; done
