#!/bin/bash
# Round 4: per-executor side reduction grid (MobileNetV2 128, ResNet-50 default) and side-stream
# LDS floor (PGDIST_SIDE_LDS_KB: caps side workgroups per CU): tests + A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4w2 && export TMPDIR=/tmp
O=gpurun_out/r4w2
timeout -k 10 500 python -u -m pytest tests/test_executor_gpu.py tests/test_resnet_executor_gpu.py tests/test_bn_lazy_gpu.py tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest.log | head -30; exit $rc; }
ab() {
  t=$1; x=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py $x > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2 3; do
  ab side384 "--steps 60 --warmup 10" PGDIST_WRED_SIDE_MNV2=0
  ab side128 "--steps 60 --warmup 10" X=1
  ab lds84 "--steps 60 --warmup 10" PGDIST_SIDE_LDS_KB=84
  ab lds56 "--steps 60 --warmup 10" PGDIST_SIDE_LDS_KB=56
done
ab rn "--model resnet50 --steps 20 --warmup 5" X=1
