#!/bin/bash
# Round 4: augmentation kernels (vectorised source staging, parallel RNG draws, composite
# separable crop-resize filters) and small-map block-output fusion (PGDIST_FUSE_BLOCK_OUT_MAXM).
# Numerics, per-op roofline, bench A/B vs ab/base (= previous commit)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/aug && export TMPDIR=/tmp
O=gpurun_out/aug
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_augment_parity_gpu.py tests/test_executor_gpu.py -x -q -k "augment or crop or jitter or rotation or random_params or contrast" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
PGDIST_AUG_EXACT=1 timeout -k 10 400 python -u -m pytest tests/test_augment_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_exact.log 2>&1
rc=$?; tail -1 $O/pytest_exact.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_exact.log | head -30; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py -x -q -k fusion --timeout 200 --timeout-method thread > $O/pytest_fuse.log 2>&1
frc=$?; tail -1 $O/pytest_fuse.log; [ $frc -eq 0 ] || grep -E "^E |Error|assert" $O/pytest_fuse.log | head -20
[ $frc -eq 0 ] || [ $frc -eq 1 ] || exit $frc
for v in new exact base fuse; do
  R=scripts/roofline.py; E="X=1"
  [ $v = base ] && R=ab/base/scripts/roofline.py
  [ $v = exact ] && E="PGDIST_AUG_EXACT=1"
  [ $v = fuse ] && E="PGDIST_FUSE_BLOCK_OUT_MAXM=25088"
  env $E timeout -k 10 300 python -u $R --out $O/roofline_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== $v $(head -1 $O/roofline_$v.txt) | $(grep ' augment ' $O/roofline_$v.txt)"
done
ab() {
  t=$1; b=$2; shift 2
  env "$@" timeout -k 10 200 python -u $b --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do
  ab base ab/base/bench.py X=1; ab new bench.py X=1
  [ $frc -eq 0 ] && { ab fuse14 bench.py PGDIST_FUSE_BLOCK_OUT_MAXM=25088; ab fuse28 bench.py PGDIST_FUSE_BLOCK_OUT_MAXM=100352; }
done
