#!/bin/bash
# Round 4: batched lazy-finalize staging (2 channels' replica-row loads in flight per thread):
# executor / kernel numerics, per-op roofline vs ab/base, bench A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/lzb && export TMPDIR=/tmp
O=gpurun_out/lzb
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_executor_teacher_forced_gpu.py tests/test_resnet_executor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest.log | head -30; exit $rc; }
for v in new base; do
  R=scripts/roofline.py; [ $v = base ] && R=ab/base/scripts/roofline.py
  timeout -k 10 300 python -u $R --out $O/roofline_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== $v $(head -1 $O/roofline_$v.txt)"
done
ab() {
  t=$1; b=$2; x=$3
  timeout -k 10 200 python -u $b $x > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do ab base ab/base/bench.py "--steps 60 --warmup 10"; ab new bench.py "--steps 60 --warmup 10"; done
for i in 1 2; do ab rn_base ab/base/bench.py "--model resnet50 --steps 20 --warmup 5"; ab rn_new bench.py "--model resnet50 --steps 20 --warmup 5"; done
