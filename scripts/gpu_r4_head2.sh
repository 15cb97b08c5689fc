#!/bin/bash
# Round 4: head A/B -- CE fused into the backward (PGDIST_HEAD_CE_FUSED) x classifier weight
# gradient on the side stream (PGDIST_HEAD_WGRAD_SIDE) against ab/base (previous commit)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/head && export TMPDIR=/tmp
O=gpurun_out/head
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k head -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ab() {
  t=$1; b=$2
  timeout -k 10 200 python -u $b --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do
  ab base ab/base/bench.py
  PGDIST_HEAD_CE_FUSED=1 PGDIST_HEAD_WGRAD_SIDE=1 ab fused_side bench.py
  PGDIST_HEAD_CE_FUSED=0 PGDIST_HEAD_WGRAD_SIDE=1 ab sep_side bench.py
  PGDIST_HEAD_CE_FUSED=1 PGDIST_HEAD_WGRAD_SIDE=0 ab fused_main bench.py
done
