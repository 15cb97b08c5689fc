#!/bin/bash
# Round 4: fp8 tile GEMMs on the block-scaled double-rate v_mfma_scale_f32_16x16x128_f8f6f4:
# numerics (both MFMA forms), bs512 bf16 / fp8 (MX on / off) benches, MFMA counter pass
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/mx && export TMPDIR=/tmp
O=gpurun_out/mx
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_fused_gpu.py tests/test_bn_lazy_gpu.py tests/test_executor_gpu.py -k "fp8 or f8" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in bf16 mx1 mx0; do
    a="--batch-size 512 --steps 20 --warmup 5"; e=1
    [ $v != bf16 ] && a="$a --fp8 1"; [ $v = mx0 ] && e=0
    PGDIST_F8_MX=$e timeout -k 10 300 python -u bench.py $a > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('bs512 $v', d['ms_per_step'], d['value'])"
  done
done
bash scripts/gpu_pmc_mfma.sh "mnv2_fp8mx_bs512:--model mobilenet_v2 --batch-size 512 --fp8 1"
