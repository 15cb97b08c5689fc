#!/bin/bash
# ResNet-50 weight-gradient (LDS-DMA) grid-size / ring-depth sweep, network totals (conv_bench wgradma)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "-" "PGDIST_WGD_TARGET=1024" "PGDIST_WGD_TARGET=2048" "PGDIST_WG_DMA_NBUF=3" "PGDIST_WGD_TARGET=1024 PGDIST_WG_DMA_NBUF=3"; do
  [ "$cfg" = "-" ] && c="" || c="$cfg"
  env $c timeout -k 10 300 python -u scripts/conv_bench.py --kinds wgradma --reps 9 > gpurun_out/wgd.txt 2>&1 || { tail -5 gpurun_out/wgd.txt; exit 1; }
  echo "== $cfg"; grep -E "c2|totals" gpurun_out/wgd.txt
done
