#!/bin/bash
# Round 6: ResNet-50 per-op roofline and MFMA counter pass of the current code
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6
timeout -k 10 400 python -u scripts/roofline.py --model resnet50 --out $O/roofline_resnet50.txt > $O/roofline_rn.log 2>&1 || { tail -20 $O/roofline_rn.log; exit 1; }
tail -25 $O/roofline_resnet50.txt
bash scripts/gpu_pmc_mfma.sh "resnet50_bs128:--model resnet50"
