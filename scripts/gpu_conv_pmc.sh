#!/bin/bash
# Counter pass over the dense-conv kernels of a few layers ($1: tag, $2: --only prefix list, $3 kinds)
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; TAG=${1:-base}; ONLY=${2:-l3.c2}; KINDS=${3:-fwd,dgradm,wgradma}
O="$R/gpurun_out/cpmc_$TAG"; mkdir -p $O
C=${PMC_COUNTERS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"}
for o in ${ONLY//,/ }; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/$o" -o run -- \
    python3 "$R/scripts/conv_bench.py" --kinds $KINDS --reps 2 --only $o > "$O/$o.log" 2>&1 || { tail -5 "$O/$o.log"; exit 1; }
  python3 "$R/scripts/pmc_table.py" "$O/$o" --filter conv > "$O/$o.csv" 2>&1; cat "$O/$o.csv"
done
