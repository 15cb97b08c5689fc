#!/bin/bash
# Round 6 check: full GPU suite (one pytest process), smoke, then same-box interleaved A/B of the
# working tree vs ab/base (scripts/ab_base.sh): MobileNetV2 default bench x3, ResNet-50 x2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 gpurun_out/abso && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
AB_TESTS= bash scripts/gpu_ab_so.sh || exit 1
A=$GRAFT_REPO_ROOT/gpurun_out/abso
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $A/rn_new_$i.json 2> $A/rn.err || { tail -20 $A/rn.err; exit 1; }
  (cd /tmp/abbase && PGDIST_AUTOBUILD=0 timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $A/rn_base_$i.json 2> $A/rn.err) || { tail -20 $A/rn.err; exit 1; }
  python -c "import json; n=json.load(open('$A/rn_new_$i.json'))['ms_per_step']; b=json.load(open('$A/rn_base_$i.json'))['ms_per_step']; print('resnet50 new', n, 'base', b)"
done
