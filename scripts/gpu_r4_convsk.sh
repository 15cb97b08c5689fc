#!/bin/bash
# Round 4: split-K for the LDS-DMA dense convs (PGDIST_CONV_SPLITK = grid target): numerics with
# splits forced everywhere they apply, ResNet-50 executor tests, per-op roofline, bench A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/csk && export TMPDIR=/tmp
O=gpurun_out/csk
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_off.log 2>&1
rc=$?; tail -1 $O/pytest_off.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest_off.log | head -30; exit $rc; }
PGDIST_CONV_SPLITK=100000 timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_on.log 2>&1
rc=$?; tail -1 $O/pytest_on.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest_on.log | head -30; exit $rc; }
for v in 0 512 1024; do
  PGDIST_CONV_SPLITK=$v timeout -k 10 300 python -u scripts/roofline.py --model resnet50 --iters 10 --out $O/roofline_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== splitk=$v $(head -1 $O/roofline_$v.txt)"
done
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do ab off PGDIST_CONV_SPLITK=0; ab sk512 PGDIST_CONV_SPLITK=512; ab sk1024 PGDIST_CONV_SPLITK=1024; done
