#!/bin/bash
# MFMA activity pass (kernel-trace + counters only) for MobileNetV2 and ResNet-50 bench steps.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc_mfma"
rm -rf "$R/gpurun_out/pmc_mfma/"*
C="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for m in mobilenet_v2 resnet50; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_mfma/$m" -o run -- python3 "$R/bench.py" --model $m --steps 2 --warmup 1 > "$R/gpurun_out/pmc_mfma/$m.log" 2>&1
  rc=$?; echo "$m rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_mfma/$m.log"; exit $rc; fi
done
