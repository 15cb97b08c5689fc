#!/bin/bash
# depthwise dgrad ring depth per variant: fused dgrad+wgrad (PGDIST_DW_DDEPTH_WG) and plain stride-1 (PGDIST_DW_DDEPTH_S1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bn_fused_gpu.py -k "dw" > $O/dd_tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/dd_tests.log | head -20; tail -3 $O/dd_tests.log; exit 1; }
tail -1 $O/dd_tests.log
i=0
for cfg in "X=1" "PGDIST_DW_DDEPTH_WG=4" "PGDIST_DW_DDEPTH_WG=5" "PGDIST_DW_DDEPTH_S1=4"; do
  env $cfg timeout -k 10 300 python -u scripts/roofline.py --out $O/dd$i.txt > $O/dd$i.log 2>&1 || { tail -5 $O/dd$i.log; exit 1; }
  echo "== dd$i $cfg $(head -1 $O/dd$i.txt)"; grep -E "^main  dw_dgrad" $O/dd$i.txt
  i=$((i+1))
done
run() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do run d3 X=1; run wg4 PGDIST_DW_DDEPTH_WG=4; run wg5 PGDIST_DW_DDEPTH_WG=5; done
