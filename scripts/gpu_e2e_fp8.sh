#!/bin/bash
# Convergence of the fp8 forward path against bf16: the same 1-GPU job (gpu128 preset,
# CIFAR-shaped synthetic data, native HIP backend) with --precision bf16 and fp8.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EPOCHS=${EPOCHS:-3}
for prec in bf16 fp8; do
  timeout -k 10 600 python train.py --preset gpu128 --data synthetic --epochs $EPOCHS --precision $prec \
    --save-path gpurun_out/best_e2e_$prec.pth > gpurun_out/e2e_$prec.log 2>&1
  rc=$?
  echo "== $prec rc=$rc"; grep -v amdgpu.ids gpurun_out/e2e_$prec.log | tail -8
  [ $rc -ne 0 ] && exit $rc
done
exit 0
