#!/bin/bash
# Full GPU test suite (one pytest process) + smoke
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_full.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_full.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
