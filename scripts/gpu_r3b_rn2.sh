#!/bin/bash
# ResNet-50 lazy BN finalize: tests (reported, not fatal), bench A/B (lazy / launch), step trace
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out; R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_resnet_executor_gpu.py \
  tests/test_conv_gpu.py > $O/rn2_tests.log 2>&1
rc=$?
grep -E "FAILED|Error|assert " $O/rn2_tests.log | head -20; tail -3 $O/rn2_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for cfg in "PGDIST_BN_LAZY=1" "PGDIST_BN_LAZY=0" "PGDIST_RN_XMASK=0" "PGDIST_BN_LAZY=1" "PGDIST_BN_LAZY=0" "PGDIST_RN_XMASK=0"; do
  env $cfg timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn2_b.json 2> $O/rn2_b.err || { tail -20 $O/rn2_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rn2_b.json')); print('$cfg', d['ms_per_step'], d['value'])"
done
rm -rf $O/prof_rn2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_rn2" -o run --output-format csv -- python3 "$R/bench.py" --model resnet50 --steps 5 --warmup 3 > "$R/$O/prof_rn2.log" 2>&1) || { echo "rocprof failed"; exit 6; }
python scripts/timeline.py $O/prof_rn2/run_kernel_trace.csv adam > $O/timeline_rn2.txt 2>&1; head -60 $O/timeline_rn2.txt
