#!/bin/bash
# ResNet-50 native path: conv kernel tests, then an isolated (no side stream) kernel profile
# analysed per conv layer (scripts/analyze_resnet_trace.py), then the bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-rn}
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 4 --warmup 3 --side-stream 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed"; exit 5; }
cd $GRAFT_REPO_ROOT && python scripts/analyze_resnet_trace.py gpurun_out/prof_${TAG}/run_kernel_trace.csv > gpurun_out/${TAG}_analysis.txt
grep -v "^  l" gpurun_out/${TAG}_analysis.txt | grep -v Cijk | head -24
timeout -k 10 200 python bench.py --model resnet50 --steps 10 --warmup 5 2>/dev/null
