#!/bin/bash
# Native communicator on the GPU: comm + DDP tests, then every GPU test, comm microbenchmark, 1-GPU bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_comm.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_comm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/comm_bench.py --out gpurun_out/comm_microbench.txt > gpurun_out/comm_bench.log 2>&1
rc=$?; tail -40 gpurun_out/comm_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 4; }
cat gpurun_out/bench_default.json
