#!/bin/bash
# Round 4 E: pw_tile shape rule vs the grid-size heuristic vs all-128x64, in the replayed step
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "pw" -x -q --timeout 120 --timeout-method thread > $O/pytest_pw.log 2>&1
rc=$?; tail -2 $O/pytest_pw.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_pw.log | head -30; exit $rc; }
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do ab rule X=1; ab heur PGDIST_TILE_RULE=0; ab all128x64 PGDIST_TILE_FORCE=128x64; done
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_rule.txt > $O/roofline_rule.log 2>&1 || { tail -20 $O/roofline_rule.log; exit 1; }
head -1 $O/roofline_rule.txt; grep -E "^main  pw_gemm|^total" $O/roofline_rule.txt
