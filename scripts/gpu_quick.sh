cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())"
for e in PGDIST_NOOP=1 PGDIST_SIDE_PRIO=-1 PGDIST_NOOP=1 PGDIST_SIDE_PRIO=-1; do
  env $e timeout -k 10 120 python bench.py --steps 30 --warmup 10 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail gpurun_out/sw.err; exit 5; }
  echo "$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json)"
done
for e in PGDIST_NOOP=1 PGDIST_SIDE_PRIO=-1; do
  env $e timeout -k 10 120 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail gpurun_out/sw.err; exit 5; }
  echo "resnet $e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json)"
done
