#!/bin/bash
# ResNet-50: stem wgrad on the main stream, batched side reductions: tests + A/B + trace
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out; R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_resnet_executor_gpu.py \
  > $O/rn3_tests.log 2>&1
rc=$?
grep -E "FAILED|Error|assert " $O/rn3_tests.log | head -20; tail -3 $O/rn3_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for cfg in "-" "PGDIST_RN_STEM_MAIN=0" "PGDIST_RED_BATCH=0" "-" "PGDIST_RN_STEM_MAIN=0" "PGDIST_RED_BATCH=0"; do
  [ "$cfg" = "-" ] && c="" || c="$cfg"
  env $c timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn3_b.json 2> $O/rn3_b.err || { tail -20 $O/rn3_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rn3_b.json')); print('${cfg}', d['ms_per_step'], d['value'])"
done
rm -rf $O/prof_rn3
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_rn3" -o run --output-format csv -- python3 "$R/bench.py" --model resnet50 --steps 5 --warmup 3 > "$R/$O/prof_rn3.log" 2>&1) || { echo "rocprof failed"; exit 6; }
python scripts/timeline.py $O/prof_rn3/run_kernel_trace.csv adam > $O/timeline_rn3.txt 2>&1; grep -A12 "longest gaps" $O/timeline_rn3.txt | head -30; grep "stream" $O/timeline_rn3.txt
