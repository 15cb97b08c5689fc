#!/bin/bash
# Round 6 final validation, part A: full GPU suite + smoke, three default bench runs (the driver's
# command line), ResNet-50 bench, per-op roofline, kernel-trace timeline of the bench step
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6final && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6final
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py > $O/bench_$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cat $O/bench_$i.json
done
timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_resnet50.json 2> $O/bench_rn.err || { tail -20 $O/bench_rn.err; exit 1; }
cat $O/bench_resnet50.json
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_mnv2.txt > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
grep -E "^total" $O/roofline_mnv2.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/timeline_mnv2.txt 2>&1; head -3 $O/timeline_mnv2.txt
