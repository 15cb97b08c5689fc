#!/bin/bash
# Round 6: ResNet-50 small kernels (branch-free max-pool backward, batched column sum, dgrad weight
# transposes on the side stream during the forward): tests, then same-box A/B vs ab/base
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 gpurun_out/abso && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_rn2.log 2>&1
rc=$?; tail -2 $O/pytest_rn2.log; grep -E "FAILED|ERROR" $O/pytest_rn2.log | head -5; [ $rc -ne 0 ] && exit $rc
A=$GRAFT_REPO_ROOT/gpurun_out/abso
rm -rf /tmp/abbase && cp -r ab/base /tmp/abbase || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $A/rn_new_$i.json 2> $A/rn.err || { tail -20 $A/rn.err; exit 1; }
  (cd /tmp/abbase && PGDIST_AUTOBUILD=0 timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $A/rn_base_$i.json 2> $A/rn.err) || { tail -20 $A/rn.err; exit 1; }
  python -c "import json; n=json.load(open('$A/rn_new_$i.json'))['ms_per_step']; b=json.load(open('$A/rn_base_$i.json'))['ms_per_step']; print('resnet50 new', n, 'base', b)"
done
