#!/bin/bash
# Round 6 (b): dwx_fwd kernel tests, executor tests, then same-box A/B of the working tree vs ab/base
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py::test_dwx_fwd -x -q --timeout 120 --timeout-method thread > $O/pytest_b1.log 2>&1
rc=$?; tail -3 $O/pytest_b1.log; grep -E "FAILED|ERROR|assert" $O/pytest_b1.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_executor_gpu.py tests/test_executor_teacher_forced_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_b2.log 2>&1
rc=$?; tail -3 $O/pytest_b2.log; grep -E "FAILED|ERROR" $O/pytest_b2.log | head; [ $rc -ne 0 ] && exit $rc
AB_TESTS= bash scripts/gpu_ab_so.sh || exit 1
