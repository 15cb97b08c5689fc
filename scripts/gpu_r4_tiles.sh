#!/bin/bash
# Round 4: small-M pointwise GEMM tile sweep -- per-op isolated roofline with every pw_tile launch
# forced onto one tile shape (PGDIST_TILE_FORCE), plus the default heuristic
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4t && export TMPDIR=/tmp
O=gpurun_out/r4t
for f in default 128x128 64x128 128x64 64x64; do
  if [ $f = default ]; then E="X=1"; else E="PGDIST_TILE_FORCE=$f"; fi
  env $E timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$f.txt > $O/roofline_$f.log 2>&1 || { tail -20 $O/roofline_$f.log; exit 1; }
  echo "== $f $(head -1 $O/roofline_$f.txt)"
done
