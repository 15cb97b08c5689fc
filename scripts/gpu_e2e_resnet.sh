#!/bin/bash
# End-to-end ResNet-50 (BASELINE config 4 model) through the same trainer on one MI355X:
# CIFAR-10-shaped synthetic data (50k / 10k, GPU augmentation to 224x224), native
# dense-conv executor, eval every epoch, best + full checkpoints.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EPOCHS=${EPOCHS:-2}
timeout -k 10 900 python train.py --preset gpu128 --model resnet50 --data synthetic --epochs $EPOCHS \
  --save-path /tmp/best_e2e_resnet50.pth --ckpt-dir /tmp/ck_resnet50 > gpurun_out/e2e_resnet50.log 2>&1
rc=$?
tail -12 gpurun_out/e2e_resnet50.log
exit $rc
