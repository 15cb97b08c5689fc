#!/bin/bash
# planted kernel-family gradient bugs on synthetic-hard (20 epochs each): all depthwise / all 1x1
# weight gradients zeroed (a broken dw_wgrad / pw_wgrad kernel)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/e2e4 && export TMPDIR=/tmp
O=gpurun_out/e2e4
for bug in @dw @pw; do
  PGDIST_FAULT_ZERO_GRAD=$bug timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic-hard --epochs 20 \
    --seed 1 --save-path $O/best_bug.pth > $O/gpu128_hard_20ep_bug_${bug#@}.log 2>&1 || { tail -10 $O/gpu128_hard_20ep_bug_${bug#@}.log; exit 1; }
  echo "== bug $bug"; grep -E "^Epoch" $O/gpu128_hard_20ep_bug_${bug#@}.log | awk '{print $NF}' | tr '\n' ' '; echo
done
