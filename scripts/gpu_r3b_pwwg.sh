#!/bin/bash
# MobileNetV2 per-op roofline under different side-stream weight-gradient settings
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pwwg && export TMPDIR=/tmp
i=0
for cfg in "X=1" "PGDIST_PWWG_WGS=2048" "PGDIST_PWWG_MINROWS=256" "PGDIST_PWWG_WGS=2048 PGDIST_PWWG_MINROWS=256" "PGDIST_PWWG_WGS=512" "PGDIST_DW_WROWS=14" "PGDIST_DW_WROWS=56"; do
  env $cfg timeout -k 10 300 python -u scripts/roofline.py --out gpurun_out/pwwg/cfg$i.txt > gpurun_out/pwwg/cfg$i.log 2>&1 || { tail -5 gpurun_out/pwwg/cfg$i.log; exit 1; }
  echo "== cfg$i $cfg"; head -1 gpurun_out/pwwg/cfg$i.txt; grep -E "side  (pw|dw)_wgrad  " gpurun_out/pwwg/cfg$i.txt
  i=$((i+1))
done
