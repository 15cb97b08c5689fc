#!/bin/bash
# conv kernel iteration: numerics tests of the dense convs, per-layer A/B timing, ResNet-50 bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/conv && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py} -x -q --timeout 120 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/conv/tests.log 2>&1
rc=$?; tail -3 gpurun_out/conv/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/conv/tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/conv_bench.py ${BENCH_ARGS:---glds 0,2,3 --kinds fwd,fwdbn} > gpurun_out/conv/bench.txt 2>&1 || { tail -20 gpurun_out/conv/bench.txt; exit 3; }
cat gpurun_out/conv/bench.txt
[ -n "$NO_RN" ] && exit 0
for m in ${RN_MODES:-0 2}; do
  PGDIST_CONV_GLDS=$m timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/conv/rn$m.json 2>gpurun_out/conv/rn$m.err || { tail -5 gpurun_out/conv/rn$m.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/conv/rn$m.json')); print('resnet50 glds=$m', d['ms_per_step'], 'ms', d['value'], 'img/s')"
done
