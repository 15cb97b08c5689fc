#!/bin/bash
# same-box A/B: depthwise dgrad at >= 3 waves/SIMD (in-tree, PGDIST_DW_DGRAD_WPE=3) vs unconstrained (ab/ copy)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "dw" > $O/ab2_tests.log 2>&1 || { grep -E "FAILED|Error" $O/ab2_tests.log | head; tail -3 $O/ab2_tests.log; exit 1; }
tail -1 $O/ab2_tests.log
run() {
  d=$1; t=$2
  (cd $d && timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/ab2_b.json 2> $O/ab2_b.err) || { tail -20 $O/ab2_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab2_b.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do run . "wpe3"; run ab "wpe1"; done
timeout -k 10 300 python -u scripts/roofline.py --out $O/ab2_roof3.txt > /dev/null 2>&1 && grep -E "dw_dgrad  " $O/ab2_roof3.txt | tail -3
(cd ab && timeout -k 10 300 python -u scripts/roofline.py --out $O/ab2_roof1.txt > /dev/null 2>&1) && grep -E "dw_dgrad  " $O/ab2_roof1.txt | tail -3
