#!/bin/bash
# Round 4: per-op roofline of the bs512 step, bf16 vs fp8 forward GEMMs (where fp8 loses)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/fp8r && export TMPDIR=/tmp
O=gpurun_out/fp8r
for v in 0 1; do
  timeout -k 10 400 python -u scripts/roofline.py --batch 512 --fp8 $v --iters 10 --out $O/roofline_fp8_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== fp8=$v $(head -1 $O/roofline_fp8_$v.txt)"
done
