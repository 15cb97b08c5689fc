#!/bin/bash
# Round 5: fused inverted-residual block forward + communicator failure handling -- numerics /
# fault tests, bench A/B (fused vs three launches), per-op roofline of the fused step
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5ir && export TMPDIR=/tmp
O=gpurun_out/r5ir
timeout -k 10 500 python -u -m pytest tests/test_irblock_gpu.py tests/test_executor_teacher_forced_gpu.py tests/test_comm_watchdog_gpu.py -x -v -rP --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -20; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/fused_$i.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  PGDIST_IR_FUSE=0 timeout -k 10 200 python -u bench.py > $O/unfused_$i.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; a=json.load(open('$O/fused_$i.json')); b=json.load(open('$O/unfused_$i.json')); print('fused', a['ms_per_step'], 'unfused', b['ms_per_step'])"
done
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline.txt > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
grep -E "ir_fwd|total" $O/roofline.txt | tail -20
timeout -k 10 500 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py tests/test_bench_gpu.py -x -q --timeout 240 --timeout-method thread > $O/comm_tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/comm_tests.log | tail -10; exit $rc
