#!/bin/bash
# Round 4: per-op cost of the lazy BN finalize in the consumers -- roofline with the finalize
# launches (PGDIST_BN_LAZY=0) vs lazy (default)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/lazy && export TMPDIR=/tmp
O=gpurun_out/lazy
for v in 1 0; do
  PGDIST_BN_LAZY=$v timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== lazy=$v $(head -1 $O/roofline_$v.txt)"
done
