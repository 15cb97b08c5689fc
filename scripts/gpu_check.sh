#!/bin/bash
# GPU validation: all GPU tests, native bench, rocprofv3 kernel stats.
# Stops at the first crash / timeout (exit codes other than 0/1 from pytest).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-30}
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed/timed out; stopping"; exit $rc; fi
[ -n "$SKIP_BENCH" ] && exit $rc
timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 > gpurun_out/bench_hip.json 2> gpurun_out/bench_hip.err || { echo "bench failed"; tail -20 gpurun_out/bench_hip.err; exit 4; }
cat gpurun_out/bench_hip.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_hip" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 --graph 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_hip.log" 2>&1
echo "rocprof rc=$?"
exit $rc
