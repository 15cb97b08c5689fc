cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_resnet_executor_gpu.py tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rn_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/rn_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rn_bench.json 2> gpurun_out/rn_bench.err || { echo bench failed; tail -20 gpurun_out/rn_bench.err; exit 4; }
cat gpurun_out/rn_bench.json
