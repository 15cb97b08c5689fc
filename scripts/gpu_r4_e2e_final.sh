#!/bin/bash
# Round 4: 20-epoch synthetic-hard gpu128 run on the final code (same seed as run 1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/e2ef && export TMPDIR=/tmp
O=gpurun_out/e2ef
timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic-hard --epochs 20 --seed 1 \
  --save-path $O/best.pth > $O/hard_20ep.log 2>&1 || { tail -10 $O/hard_20ep.log; exit 1; }
grep -E "^Epoch|Best|Total" $O/hard_20ep.log | tail -5
