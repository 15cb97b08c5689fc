#!/bin/bash
# per-shape DMA wgrad config + one-stage LDS for one-k-step convs: tests, bench A/B, tables
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py > $O/rn4_tests.log 2>&1 || { grep -E "FAILED|Error" $O/rn4_tests.log | head; tail -5 $O/rn4_tests.log; exit 1; }
tail -1 $O/rn4_tests.log
for cfg in "-" "PGDIST_CONV_1STAGE=0" "-" "PGDIST_CONV_1STAGE=0"; do
  [ "$cfg" = "-" ] && c="" || c="$cfg"
  env $c timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn4_b.json 2> $O/rn4_b.err || { tail -20 $O/rn4_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rn4_b.json')); print('$cfg', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,dgradm,wgradma --reps 7 > $O/rn4_conv.txt 2>&1 && grep totals $O/rn4_conv.txt
PGDIST_CONV_1STAGE=0 timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,dgradm --reps 7 > $O/rn4_conv0.txt 2>&1 && grep totals $O/rn4_conv0.txt
