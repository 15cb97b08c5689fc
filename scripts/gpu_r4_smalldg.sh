#!/bin/bash
# Round 4: round-aware small-map depthwise dgrad geometry (tall strips on): numerics, isolated
# per-layer times, bench A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/sdg && export TMPDIR=/tmp
O=gpurun_out/sdg
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dw_" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
rm -f $O/dw.txt
for v in "0 12" "1 4" "1 12" "1 24"; do
  set -- $v
  echo "== PGDIST_DW_SMALL_DGRAD=$1 PGDIST_DW_FIX=$2" >> $O/dw.txt
  PGDIST_DW_SMALL_DGRAD=$1 PGDIST_DW_FIX=$2 timeout -k 10 200 python -u scripts/dw_bench.py --kinds dgrad --reps 30 >> $O/dw.txt 2>&1 || { tail -20 $O/dw.txt; exit 1; }
done
grep -E "==|H= +(7|14) s=1|network" $O/dw.txt
for i in 1 2 3; do
  for v in 0 1; do
    PGDIST_DW_SMALL_DGRAD=$v timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('small_dgrad $v', d['ms_per_step'], d['value'])"
  done
done
