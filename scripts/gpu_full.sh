#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), the default bench and a kernel-stats profile.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 4; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --model resnet50 > gpurun_out/bench_resnet.json 2> gpurun_out/bench_resnet.err || { tail gpurun_out/bench_resnet.err; exit 5; }
cat gpurun_out/bench_resnet.json
timeout -k 10 300 python bench.py --batch-size 512 --fp8 1 > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err || { tail gpurun_out/bench_fp8.err; exit 6; }
cat gpurun_out/bench_fp8.json
