#!/bin/bash
# Round 4: fp8 layer policy (e4m3 only for K >= 64; block-output fusion where the consumer is bf16):
# fp8 tests, bs512 bf16 vs fp8 back to back
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/fp8p && export TMPDIR=/tmp
O=gpurun_out/fp8p
timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_kernels_gpu.py -x -q -k "fp8" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest.log | head -30; exit $rc; }
ab() {
  t=$1; x=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py $x > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do
  ab bf16 "--batch-size 512 --steps 20 --warmup 5" X=1
  ab fp8_k64 "--batch-size 512 --fp8 1 --steps 20 --warmup 5" X=1
  ab fp8_all "--batch-size 512 --fp8 1 --steps 20 --warmup 5" PGDIST_FP8_MIN_K=0
done
