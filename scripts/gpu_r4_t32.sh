#!/bin/bash
# Round 4: 32-row pw_tile tiles for the long-K small-M GEMMs (PGDIST_TILE_RULE=2): numerics with
# every pw_tile launch forced onto 32x64 / 32x128, per-op roofline, bench A/B on one box
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/t32 && export TMPDIR=/tmp
O=gpurun_out/t32
for f in 32x64 32x128; do
  PGDIST_TILE_FORCE=$f timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pw_" --timeout 200 --timeout-method thread > $O/pytest_$f.log 2>&1
  rc=$?; tail -1 $O/pytest_$f.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_$f.log | head -30; exit $rc; }
done
for r in 1 2; do
  PGDIST_TILE_RULE=$r timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$r.txt > $O/roofline_$r.log 2>&1 || { tail -20 $O/roofline_$r.log; exit 1; }
  echo "== rule=$r $(head -1 $O/roofline_$r.txt)"
done
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do ab rule1 PGDIST_TILE_RULE=1; ab rule2 PGDIST_TILE_RULE=2; done
