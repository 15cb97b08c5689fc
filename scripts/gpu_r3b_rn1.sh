#!/bin/bash
# ResNet-50: replica-row BN statistics + space-to-depth stem: tests, bench A/B, roofline
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_executor_gpu.py > $O/rn1_tests.log 2>&1 || { grep -E "FAILED|Error|error" $O/rn1_tests.log | head -30; tail -30 $O/rn1_tests.log; exit 1; }
tail -3 $O/rn1_tests.log
for cfg in "PGDIST_RN_STEM=s2d" "PGDIST_RN_STEM=direct" "PGDIST_RN_STEM=s2d"; do
  env $cfg timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn1_b.json 2> $O/rn1_b.err || { tail -20 $O/rn1_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rn1_b.json')); print('$cfg', d['ms_per_step'], d['value'])"
done
timeout -k 10 400 python -u scripts/roofline.py --model resnet50 --out $O/roofline_rn1.txt > $O/roofline_rn1.log 2>&1 \
  || { tail -20 $O/roofline_rn1.log; exit 1; }
tail -24 $O/roofline_rn1.txt
