#!/bin/bash
# Round 4 H: next-batch augmentation prefetch beside the forward (side stream idle) vs beside the backward
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_augment_parity_gpu.py tests/test_trainer.py -x -q --timeout 200 --timeout-method thread > $O/pytest_h.log 2>&1
rc=$?; tail -2 $O/pytest_h.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_h.log | head -30; exit $rc; }
ab() {
  t=$1; b=$2; shift 2
  env "$@" timeout -k 10 200 python -u $b --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do ab base ab/base/bench.py X=1; ab fwd bench.py X=1; ab bwd bench.py PGDIST_AUG_PREFETCH_AT=backward; done
