#!/bin/bash
# Round 4: bs512 bf16 vs fp8 (K >= 64 layer policy) on synthetic-hard, 8 epochs, same seed; plus
# fp8 on every 1x1 conv for reference
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/e2e8 && export TMPDIR=/tmp
O=gpurun_out/e2e8
for p in bf16 fp8 fp8all; do
  prec=$p; E="X=1"; [ $p = fp8all ] && { prec=fp8; E="PGDIST_FP8_MIN_K=0"; }
  env $E timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic-hard --epochs 8 --batch-size 512 --precision $prec \
    --seed 1 --save-path $O/best_$p.pth > $O/hard_bs512_${p}_8ep.log 2>&1 || { tail -10 $O/hard_bs512_${p}_8ep.log; exit 1; }
  echo "== $p"; grep -E "^Epoch|Best|Total" $O/hard_bs512_${p}_8ep.log | tail -4
done
