#!/bin/bash
# pw_bwd change: focused kernel tests, then bench + roofline ($1 tag)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-pw}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_lazy_gpu.py tests/test_executor_teacher_forced_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 4; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python -u scripts/roofline.py --out gpurun_out/roofline_$TAG.txt > gpurun_out/roofline_$TAG.log 2>&1 || exit 5
tail -24 gpurun_out/roofline_$TAG.log
