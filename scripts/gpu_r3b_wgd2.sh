#!/bin/bash
# full per-layer wgrad tables for the candidate DMA-wgrad configurations
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/wgd && export TMPDIR=/tmp
i=0
for cfg in "-" "PGDIST_WGD_TARGET=1024" "PGDIST_WG_DMA_MK=32 PGDIST_WG_DMA_NBUF=3" "PGDIST_WG_DMA_MK=32 PGDIST_WG_DMA_NBUF=3 PGDIST_WGD_TARGET=1024" "PGDIST_WGD_TARGET=768"; do
  [ "$cfg" = "-" ] && c="" || c="$cfg"
  env $c timeout -k 10 300 python -u scripts/conv_bench.py --kinds wgradma --reps 7 > gpurun_out/wgd/cfg$i.txt 2>&1 || { tail -5 gpurun_out/wgd/cfg$i.txt; exit 1; }
  echo "== cfg$i $cfg"; grep totals gpurun_out/wgd/cfg$i.txt
  i=$((i+1))
done
