#!/bin/bash
# Round 6 closing validation (after the ResNet-50 BN / materialisation changes): full GPU suite +
# smoke, three default bench runs, two ResNet-50 bench runs, ResNet-50 roofline, kernel-trace
# timeline and MFMA counters.  Each GPU step has its own limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6d && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6d
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py > $O/bench_$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cat $O/bench_$i.json
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_resnet50_$i.json 2> $O/bench_rn.err || { tail -20 $O/bench_rn.err; exit 1; }
  cat $O/bench_resnet50_$i.json
done
timeout -k 10 300 python -u scripts/roofline.py --model resnet50 --out $O/roofline_resnet50.txt > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
grep -E "^total" $O/roofline_resnet50.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/timeline_resnet50.txt 2>&1; head -3 $O/timeline_resnet50.txt
bash scripts/gpu_pmc_mfma.sh "resnet50_bs128:--model resnet50"
