#!/bin/bash
# New parity tests (augmentation render, teacher-forced executor, serving floor).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_augment_parity_gpu.py tests/test_executor_teacher_forced_gpu.py tests/test_serve.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_parity.log | tail -40; tail -3 gpurun_out/pytest_parity.log; exit $rc
