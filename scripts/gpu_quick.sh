cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_serve.py -m gpu -x -q --timeout 120 --timeout-method thread -k "head or graph_modes or loss_decreases or step_matches or serve or predict" > gpurun_out/t_q.log 2>&1; rc=$?; tail -3 gpurun_out/t_q.log; [ $rc -eq 0 ] || { grep -B5 -A25 "Error\|assert" gpurun_out/t_q.log | head -60; exit $rc; }
for g in 0 2 0 2; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 10 --graph $g > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail gpurun_out/sw.err; exit 5; }
  echo "graph=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json)"
done
