#!/bin/bash
# same-box A/B: packed epilogue stores (in-tree) vs per-element stores (ab/ copy built with
# PGDIST_PACKED_EPI=0); wide forward expand tiles on/off (PGDIST_PW_WIDE_FWD)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_executor_gpu.py > $O/ab_tests.log 2>&1 || { grep -E "FAILED|Error" $O/ab_tests.log | head; tail -3 $O/ab_tests.log; exit 1; }
tail -1 $O/ab_tests.log
run() {  # dir tag env...
  d=$1; t=$2; shift 2
  (cd $d && env "$@" timeout -k 10 200 python -u bench.py $BA > $O/ab_b.json 2> $O/ab_b.err) || { tail -20 $O/ab_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab_b.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do
  BA="--steps 40 --warmup 10"
  run . "mnv2 packed wide" X=1
  run . "mnv2 packed narrow" PGDIST_PW_WIDE_FWD=0
  run ab "mnv2 plain wide" X=1
  run ab "mnv2 plain narrow" PGDIST_PW_WIDE_FWD=0
  BA="--model resnet50 --steps 20 --warmup 5"
  run . "rn50 packed" X=1
  run ab "rn50 plain" X=1
done
timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,dgradm --reps 7 > $O/ab_conv_packed.txt 2>&1 && grep totals $O/ab_conv_packed.txt
(cd ab && timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,dgradm --reps 7 > $O/ab_conv_plain.txt 2>&1) && grep totals $O/ab_conv_plain.txt
