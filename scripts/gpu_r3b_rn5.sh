#!/bin/bash
# packed epilogue C-tile writes: conv + ResNet tests, conv tables, ResNet + MobileNetV2 bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py > $O/rn5_tests.log 2>&1 || { grep -E "FAILED|Error" $O/rn5_tests.log | head; tail -5 $O/rn5_tests.log; exit 1; }
tail -1 $O/rn5_tests.log
timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,dgradm --reps 7 > $O/rn5_conv.txt 2>&1 && grep totals $O/rn5_conv.txt
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn5_b.json 2> $O/rn5_b.err || { tail -20 $O/rn5_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rn5_b.json')); print('rn50', d['ms_per_step'], d['value'])"
done
timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/rn5_mb.json 2> $O/rn5_mb.err || { tail -20 $O/rn5_mb.err; exit 1; }
python -c "import json; d=json.load(open('$O/rn5_mb.json')); print('mnv2', d['ms_per_step'], d['value'])"
