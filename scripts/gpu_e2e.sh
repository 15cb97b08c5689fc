#!/bin/bash
# End-to-end job on one MI355X: the reference's 1-GPU mode (cifar10_128batch.py preset)
# on CIFAR-10-shaped synthetic data (no dataset download on the box): 50k train / 10k test
# uint8 32x32x3 images, GPU augmentation to 224x224, native HIP backend, eval every epoch.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EPOCHS=${EPOCHS:-3}
timeout -k 10 900 python train.py --preset gpu128 --data synthetic --epochs $EPOCHS \
  --save-path gpurun_out/best_e2e.pth > gpurun_out/e2e.log 2>&1
rc=$?
tail -20 gpurun_out/e2e.log
exit $rc
