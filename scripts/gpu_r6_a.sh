#!/bin/bash
# Round 6 (a): tests of the new code (watchdog poison-only, overlapped BN broadcast, ResNet lazy BN,
# pw_bwd Y recompute kernel + executor), then same-box A/B of the working tree vs ab/base
# (scripts/ab_base.sh), then the world-1-forced DP step with / without the BN broadcast
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py::test_pw_bwd_fused tests/test_executor_gpu.py tests/test_executor_teacher_forced_gpu.py tests/test_comm_watchdog_gpu.py tests/test_ddp_gpu.py tests/test_resnet_executor_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_a.log 2>&1
rc=$?; tail -3 $O/pytest_a.log; grep -E "FAILED|ERROR" $O/pytest_a.log | head; [ $rc -ne 0 ] && exit $rc
AB_TESTS= bash scripts/gpu_ab_so.sh || exit 1
for i in 1 2; do
  for b in 0 1; do
    PGDIST_FORCE_DDP=1 timeout -k 10 200 python -u bench.py --bn-broadcast $b > $O/bnb_${b}_$i.out 2> $O/bnb.err || { tail -20 $O/bnb.err; exit 1; }
    grep '^{' $O/bnb_${b}_$i.out | tail -1 > $O/bnb_${b}_$i.json
    python -c "import json; d=json.load(open('$O/bnb_${b}_$i.json')); print('bn_broadcast', $b, d['ms_per_step'])"
  done
done
