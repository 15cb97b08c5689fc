#!/bin/bash
# Round 4: plain stride-1 depthwise dgrad compiled for 4 waves per SIMD (PGDIST_DW_DGRAD_W4=1:
# 128 VGPRs + 52 B scratch) vs 3 (139 VGPRs)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/w4 && export TMPDIR=/tmp
O=gpurun_out/w4
timeout -k 10 300 env PGDIST_DW_DGRAD_W4=1 python -u -m pytest tests/test_kernels_gpu.py -k "dw_dgrad or dw_tall" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
rm -f $O/dw.txt
for e in 0 1; do
  echo "== PGDIST_DW_DGRAD_W4=$e" >> $O/dw.txt
  PGDIST_DW_DGRAD_W4=$e timeout -k 10 200 python -u scripts/dw_bench.py --kinds dgrad --reps 30 >> $O/dw.txt 2>&1 || { tail -20 $O/dw.txt; exit 1; }
done
grep -E "==|s=1|network" $O/dw.txt
for i in 1 2 3; do
  for e in 0 1; do
    PGDIST_DW_DGRAD_W4=$e timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('w4 $e', d['ms_per_step'], d['value'])"
  done
done
