#!/bin/bash
# Round 4: fail-loud communicator (release/acquire barrier, desync detection, poisoning) on the GPU:
# comm tests, DDP tests, 2-rank bench health / fault injection, comm microbench, 1-GPU bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_comm.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" $O/pytest_comm.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_ddp.log 2>&1
rc=$?; tail -3 $O/pytest_ddp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/comm_bench.py --out $O/comm_microbench.txt > $O/comm_bench.log 2>&1
rc=$?; tail -30 $O/comm_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 4; }
cat $O/bench_default.json
