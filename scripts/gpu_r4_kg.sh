#!/bin/bash
# Round 4: two k groups (8 waves) per pw_tile workgroup (PGDIST_TILE_KG=2): numerics with the knob on
# (default and forced tiles), executor step, per-op roofline, bench A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/kg && export TMPDIR=/tmp
O=gpurun_out/kg
for f in default 64x64 32x64 128x64 64x128; do
  E="PGDIST_TILE_KG=2"; [ $f != default ] && E="PGDIST_TILE_KG=2 PGDIST_TILE_FORCE=$f"
  env $E timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pw_" --timeout 120 --timeout-method thread > $O/pytest_$f.log 2>&1
  rc=$?; tail -1 $O/pytest_$f.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest_$f.log | head -30; exit $rc; }
done
PGDIST_TILE_KG=2 timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_executor_teacher_forced_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_exe.log 2>&1
rc=$?; tail -1 $O/pytest_exe.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest_exe.log | head -30; exit $rc; }
for v in 1 2; do
  PGDIST_TILE_KG=$v timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== kg=$v $(head -1 $O/roofline_$v.txt)"
done
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do ab kg1 PGDIST_TILE_KG=1; ab kg2 PGDIST_TILE_KG=2; done
