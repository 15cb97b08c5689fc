#!/bin/bash
# full GPU suite + smoke + MobileNetV2 / ResNet-50 benches + conv tables
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > $O/full_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/full_tests.log | head -20; tail -2 $O/full_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/full_smoke.log 2>&1 || { tail -20 $O/full_smoke.log; exit 1; }
tail -1 $O/full_smoke.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/full_mb.json 2> $O/full_mb.err || { tail -20 $O/full_mb.err; exit 1; }
  python -c "import json; d=json.load(open('$O/full_mb.json')); print('mnv2', d['ms_per_step'], d['value'])"
  timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/full_rn.json 2> $O/full_rn.err || { tail -20 $O/full_rn.err; exit 1; }
  python -c "import json; d=json.load(open('$O/full_rn.json')); print('rn50', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,dgradm,wgradma --reps 7 > $O/full_conv.txt 2>&1 && grep totals $O/full_conv.txt
