cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "head or dw_" > gpurun_out/t_head.log 2>&1 && tail -3 gpurun_out/t_head.log &&
for e in PGDIST_NOOP=1 PGDIST_DW_ROWS_SMALL=4 PGDIST_DW_ROWS_SMALL=7 PGDIST_NOOP=1; do
  env $e timeout -k 10 120 python bench.py --steps 30 --warmup 10 > gpurun_out/sw.json 2> gpurun_out/sw.err || exit 5
  echo "$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json)"
done
