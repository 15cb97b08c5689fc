#!/bin/bash
# Lazy BN finalize: numerics tests, A/B bench against separate finalize launches, kernel trace.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_bn_lazy_gpu.py tests/test_executor_gpu.py tests/test_bn_fused_gpu.py \
  -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lazy.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_lazy.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_lazy.log | head -20; exit $rc; }
for mode in 1 0 1 0; do
  PGDIST_BN_LAZY=$mode timeout -k 10 300 python bench.py --steps 40 --warmup 10 > gpurun_out/bench_lazy$mode.json 2> gpurun_out/bench_lazy$mode.err || { tail gpurun_out/bench_lazy$mode.err; exit 4; }
  echo "lazy=$mode $(python -c "import json;d=json.load(open('gpurun_out/bench_lazy$mode.json'));print(d['ms_per_step'], d['value'])")"
done
timeout -k 10 300 python bench.py --batch-size 512 --fp8 1 > gpurun_out/bench_lazy_fp8.json 2> gpurun_out/bench_lazy_fp8.err || { tail gpurun_out/bench_lazy_fp8.err; exit 5; }
cat gpurun_out/bench_lazy_fp8.json
rm -rf gpurun_out/prof_lazy
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_lazy" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_lazy.log" 2>&1) || exit 6
echo prof ok
