#!/bin/bash
# ResNet-50 weight-gradient (LDS-DMA) grid-size / ring-depth / stage-rows sweep (conv_bench wgradma network totals)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "wgrad" > gpurun_out/wgd_tests.log 2>&1 || { tail -20 gpurun_out/wgd_tests.log; exit 1; }
tail -1 gpurun_out/wgd_tests.log
PGDIST_WG_DMA_MK=32 PGDIST_WG_DMA_NBUF=4 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "wgrad" > gpurun_out/wgd_tests2.log 2>&1 || { tail -20 gpurun_out/wgd_tests2.log; exit 1; }
tail -1 gpurun_out/wgd_tests2.log
for cfg in "-" "PGDIST_WGD_TARGET=1024" "PGDIST_WGD_TARGET=2048" "PGDIST_WG_DMA_NBUF=3" "PGDIST_WG_DMA_MK=32 PGDIST_WG_DMA_NBUF=4" "PGDIST_WG_DMA_MK=32 PGDIST_WG_DMA_NBUF=3" "PGDIST_WG_DMA_MK=32 PGDIST_WG_DMA_NBUF=4 PGDIST_WGD_TARGET=1024"; do
  [ "$cfg" = "-" ] && c="" || c="$cfg"
  env $c timeout -k 10 300 python -u scripts/conv_bench.py --kinds wgradma --reps 7 > gpurun_out/wgd.txt 2>&1 || { tail -5 gpurun_out/wgd.txt; exit 1; }
  echo "== $cfg"; grep -E "c2 |totals" gpurun_out/wgd.txt
done
