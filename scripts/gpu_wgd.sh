#!/bin/bash
# LDS-DMA weight gradient: numerics tests, then per-layer timings on/off
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/wgd; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k wgrad > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u scripts/conv_bench.py --kinds wgradma,matb,dgradm --reps 9 > $O/on.txt 2>&1 || { tail -20 $O/on.txt; exit 1; }
cat $O/on.txt
PGDIST_WG_DMA_NBUF=3 timeout -k 10 300 python -u scripts/conv_bench.py --kinds wgradma --reps 9 > $O/on3.txt 2>&1 || { tail -20 $O/on3.txt; exit 1; }
cat $O/on3.txt
PGDIST_WG_DMA=0 timeout -k 10 300 python -u scripts/conv_bench.py --kinds wgradma,wgrad --reps 9 > $O/off.txt 2>&1 || { tail -20 $O/off.txt; exit 1; }
cat $O/off.txt
