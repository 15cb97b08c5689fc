#!/bin/bash
# Round 4 C: prologue reordering (first operand loads / DMA rows before BN-parameter staging):
# kernel numerics, executor tests, same-box A/B against the previous commit's build (ab/base),
# then the synthetic-hard signal calibration
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_c.log 2>&1
rc=$?; tail -3 $O/pytest_c.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_c.log | head -30; exit $rc; }
ab() {
  t=$1; b=$2
  timeout -k 10 200 python -u $b --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do ab base ab/base/bench.py; ab new bench.py; done
bash scripts/gpu_r4_calib.sh
