#!/bin/bash
# pw_wgrad split floor: per-shape default (256 rows when N*K <= 200k) vs the old global 512; 128 for small weights
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do run new X=1; run old PGDIST_PWWG_MINROWS=512; run small128 PGDIST_PWWG_MINROWS_SMALL=128; run fuse112 PGDIST_DW_FUSE_MIN_H=112; done
i=0
for cfg in "X=1" "PGDIST_PWWG_MINROWS_SMALL=128" "PGDIST_PWWG_MINROWS_SMALL=128 PGDIST_PWWG_WGS=2048" "PGDIST_DW_FUSE_MIN_H=112"; do
  env $cfg timeout -k 10 300 python -u scripts/roofline.py --out $O/cfg$i.txt > $O/cfg$i.log 2>&1 || { tail -5 $O/cfg$i.log; exit 1; }
  echo "== cfg$i $cfg"; head -1 $O/cfg$i.txt; grep -E "^side  " $O/cfg$i.txt
  i=$((i+1))
done
