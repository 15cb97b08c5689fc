#!/bin/bash
# Round 4: 128-wide k steps for the long-K small-M pointwise GEMMs (PGDIST_TILE_K128 threshold):
# numerics with the knob on, per-op isolated roofline, and the bench A/B on one box
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k128 && export TMPDIR=/tmp
O=gpurun_out/k128
PGDIST_TILE_K128=256 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pw_" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
for k in 0 256; do
  PGDIST_TILE_K128=$k timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$k.txt > $O/roofline_$k.log 2>&1 || { tail -20 $O/roofline_$k.log; exit 1; }
  echo "== k128=$k $(head -1 $O/roofline_$k.txt)"
done
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do ab k0 PGDIST_TILE_K128=0; ab k256 PGDIST_TILE_K128=256; ab k512 PGDIST_TILE_K128=512; done
