cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q > gpurun_out/pytest_kernels.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_kernels.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/diag_executor.py 8 64 > gpurun_out/diag_8_64.log 2>&1; echo "diag rc=$?"
timeout -k 10 300 python scripts/diag_executor.py 16 224 > gpurun_out/diag_16_224.log 2>&1; echo "diag rc=$?"
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_hip.json 2> gpurun_out/bench_hip.err; echo "bench rc=$?"; cat gpurun_out/bench_hip.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_hip" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 --graph 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_hip.log" 2>&1; echo "prof rc=$?"
