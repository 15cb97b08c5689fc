#!/bin/bash
# calibrate the synthetic-hard class-signal strength: 10-epoch gpu128 curves
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/calib && export TMPDIR=/tmp
O=gpurun_out/calib
for sig in 0.7 1.0 1.5; do
  timeout -k 10 300 python -u train.py --preset gpu128 --data synthetic-hard --synthetic-signal $sig --epochs 10 --seed 1 \
    --save-path $O/b.pth > $O/sig_$sig.log 2>&1 || { tail -10 $O/sig_$sig.log; exit 1; }
  echo "== signal $sig"; grep -E "^Epoch" $O/sig_$sig.log | awk '{print $2, $11, $13}' | tr '\n' ' '; echo
done
