#!/bin/bash
# Round 5 final measurements: three default bench.py runs (the driver's command line), one
# ResNet-50 run, then the per-op roofline of the same build
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5final && export TMPDIR=/tmp
O=gpurun_out/r5final
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  cat $O/bench_$i.json
done
timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_resnet50.json 2> $O/bench_rn.err || { tail -20 $O/bench_rn.err; exit 1; }
cat $O/bench_resnet50.json
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline.txt > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
head -1 $O/roofline.txt; grep -E "^total" $O/roofline.txt
