#!/bin/bash
# Round 5: fused inverted-residual blocks (forward + backward) and communicator failure
# handling -- numerics / fault tests, bench A/B (fused vs three launches), per-op roofline
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5ir && export TMPDIR=/tmp
O=gpurun_out/r5ir
timeout -k 10 300 python -u -m pytest tests/test_irblock_gpu.py -x -v -rP --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 1 fwd 0; do
    PGDIST_IR_FUSE=$m timeout -k 10 200 python -u bench.py > $O/bench_${m}_$i.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  done
  python -c "import json; r={m: json.load(open('$O/bench_'+m+'_$i.json'))['ms_per_step'] for m in ('1','fwd','0')}; print('fused fwd+bwd', r['1'], 'fused fwd', r['fwd'], 'unfused', r['0'])"
done
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline.txt > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
grep -E "ir_fwd|ir_bwd|total" $O/roofline.txt | tail -24
timeout -k 10 500 python -u -m pytest tests/test_comm_watchdog_gpu.py tests/test_comm_gpu.py tests/test_ddp_gpu.py tests/test_bench_gpu.py -x -q -rP --timeout 240 --timeout-method thread > $O/comm_tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/comm_tests.log | tail -10; exit $rc
