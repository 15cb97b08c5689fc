#!/bin/bash
# occupancy-aware depthwise geometry (PGDIST_DW_GEOM bit mask: 1 fwd, 2 dgrad, 4 wgrad): tests, bench A/B, per-op rows
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "dw" > $O/dwg_tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/dwg_tests.log | head -20; tail -3 $O/dwg_tests.log; exit 1; }
tail -1 $O/dwg_tests.log
run() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do run geom0 PGDIST_DW_GEOM=0; run geom2 PGDIST_DW_GEOM=2; run geom7 PGDIST_DW_GEOM=7; done
for m in 0 1 2 4; do
  PGDIST_DW_GEOM=$m timeout -k 10 300 python -u scripts/roofline.py --out $O/dwg$m.txt > $O/dwg$m.log 2>&1 || { tail -5 $O/dwg$m.log; exit 1; }
  echo "== geom $m $(head -1 $O/dwg$m.txt)"; grep -E "^(main|side)  dw_" $O/dwg$m.txt
done
