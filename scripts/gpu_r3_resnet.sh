#!/bin/bash
# ResNet-50 (BASELINE config 4): executor tests, plan vs eager bench, per-op roofline
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_executor_gpu.py \
  > $O/rn_tests.log 2>&1 || { tail -40 $O/rn_tests.log; exit 1; }
tail -3 $O/rn_tests.log
timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn_bench_plan.json 2> $O/rn_bench_plan.err \
  || { tail -20 $O/rn_bench_plan.err; exit 1; }
cat $O/rn_bench_plan.json
PGDIST_PLAN=0 timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn_bench_eager.json 2> $O/rn_bench_eager.err \
  || { tail -20 $O/rn_bench_eager.err; exit 1; }
cat $O/rn_bench_eager.json
timeout -k 10 400 python -u scripts/roofline.py --model resnet50 --out $O/roofline_rn.txt > $O/roofline_rn.log 2>&1 \
  || { tail -20 $O/roofline_rn.log; exit 1; }
tail -40 $O/roofline_rn.txt
