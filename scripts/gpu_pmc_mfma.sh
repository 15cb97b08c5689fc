#!/bin/bash
# MFMA activity pass (kernel-trace + counters only) over bench steps; each arg is
# "tag:bench args" (default: the flagship MobileNetV2 bs128, fp8 bs512, ResNet-50 bs128)
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/pmc_mfma"; mkdir -p "$O"
C="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
[ $# -eq 0 ] && set -- "mnv2_bs128:--model mobilenet_v2" "mnv2_fp8_bs512:--model mobilenet_v2 --batch-size 512 --fp8 1" \
  "mnv2_bf16_bs512:--model mobilenet_v2 --batch-size 512" "resnet50_bs128:--model resnet50"
for spec in "$@"; do
  tag=${spec%%:*}; args=${spec#*:}
  rm -rf "$O/$tag"
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/$tag" -o run -- \
    python3 "$R/bench.py" $args --steps 2 --warmup 1 > "$O/$tag.log" 2>&1
  rc=$?; echo "$tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/$tag.log"; exit $rc; fi
  python3 "$R/scripts/mfma_summary.py" "$O/$tag" 3 "$tag: $args" | tee "$O/$tag.txt" | head -12
done
