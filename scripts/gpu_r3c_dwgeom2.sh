#!/bin/bash
# depthwise geometry model restricted to stride-1 dgrad on >= 56-row maps (default mask 2) vs off
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bn_fused_gpu.py tests/test_bn_lazy_gpu.py -k "dw" > $O/dwg2_tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/dwg2_tests.log | head -20; tail -3 $O/dwg2_tests.log; exit 1; }
tail -1 $O/dwg2_tests.log
run() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do run default X=1; run geom0 PGDIST_DW_GEOM=0; done
timeout -k 10 300 python -u scripts/roofline.py --out $O/dwgd.txt > $O/dwgd.log 2>&1 || { tail -5 $O/dwgd.log; exit 1; }
echo "== default $(head -1 $O/dwgd.txt)"; grep -E "^(main|side)  " $O/dwgd.txt
