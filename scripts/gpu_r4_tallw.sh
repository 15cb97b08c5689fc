#!/bin/bash
# Round 4: tall strips for the small-map depthwise weight gradient (side stream): numerics,
# isolated per-layer times, bench A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/tallw && export TMPDIR=/tmp
O=gpurun_out/tallw
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dw_" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
rm -f $O/dw.txt
for r in 0 14 28; do
  echo "== PGDIST_DW_TALL_W=$r" >> $O/dw.txt
  PGDIST_DW_TALL_W=$r timeout -k 10 200 python -u scripts/dw_bench.py --kinds wgrad --reps 30 >> $O/dw.txt 2>&1 || { tail -20 $O/dw.txt; exit 1; }
done
grep -E "==|H= +(7|14) s=1|network" $O/dw.txt
for i in 1 2 3; do
  for r in 0 14 28; do
    PGDIST_DW_TALL_W=$r timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('tall_w $r', d['ms_per_step'], d['value'])"
  done
done
