#!/bin/bash
# Round 6: side-stream weight gradients of the small-map stages held back until the backward
# reaches maps of >= H rows (PGDIST_SIDE_DEFER_H; 0 = off), interleaved bench runs on one box
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
PGDIST_SIDE_DEFER_H=28 timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_side.log 2>&1
rc=$?; tail -2 $O/pytest_side.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for h in 0 14 28 56; do
    PGDIST_SIDE_DEFER_H=$h timeout -k 10 200 python -u bench.py > $O/side_${h}_$i.json 2> $O/side.err || { tail -20 $O/side.err; exit 1; }
    python -c "import json; print('defer_h', $h, json.load(open('$O/side_${h}_$i.json'))['ms_per_step'])"
  done
done
