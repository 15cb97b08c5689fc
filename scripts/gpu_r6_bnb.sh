#!/bin/bash
# Round 6: new GPU tests (watchdog poison-only, overlapped BN broadcast, ResNet lazy BN), then the
# world-1-forced data-parallel step (RCCL buckets) with / without the per-step BN broadcast, interleaved
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_comm_watchdog_gpu.py tests/test_ddp_gpu.py tests/test_resnet_executor_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_bnb.log 2>&1
rc=$?; tail -3 $O/pytest_bnb.log; grep -E "FAILED|ERROR" $O/pytest_bnb.log | head; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for b in 0 1; do
    PGDIST_FORCE_DDP=1 timeout -k 10 200 python -u bench.py --bn-broadcast $b > $O/bnb_${b}_$i.json 2> $O/bnb.err || { tail -20 $O/bnb.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bnb_${b}_$i.json')); print('bn_broadcast', $b, d['ms_per_step'])"
  done
done
