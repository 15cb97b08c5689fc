#!/bin/bash
# Round 4 checkpoint A: split-K small-M pointwise GEMM + LDS-DMA pointwise wgrad (numerics, A/B
# bench), then the fail-loud communicator tests, executor / DDP tests, comm microbench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "pw" -x -q --timeout 120 --timeout-method thread > $O/pytest_pw.log 2>&1
rc=$?; tail -3 $O/pytest_pw.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_pw.log | head -30; exit $rc; }
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2; do ab new X=1; ab nosplitk PGDIST_PW_SPLITK=0; ab nodma PGDIST_PWWG_DMA=0; ab prio PGDIST_MAIN_PRIO=1; ab wgs512 PGDIST_PWWG_WGS=512; ab narrow PGDIST_PWWG_DMA_WIDE=0; done
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_comm.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" $O/pytest_comm.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exe.log 2>&1
rc=$?; tail -3 $O/pytest_exe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/comm_bench.py --out $O/comm_microbench.txt > $O/comm_bench.log 2>&1
rc=$?; tail -30 $O/comm_bench.log; [ $rc -eq 0 ] || exit $rc
