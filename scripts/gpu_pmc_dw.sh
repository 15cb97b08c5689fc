#!/bin/bash
# PMC counters of the depthwise kernels (scripts/dw_bench.py, kinds from $1, default fwd), one pass per group.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; KINDS=${1:-fwd}; TAG=${2:-base}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE"
P2="TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TD_TD_BUSY TD_TC_STALL SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P -d "$R/gpurun_out/pmc_dw_${TAG}_$i" -o run --output-format csv -- python3 "$R/scripts/dw_bench.py" --reps 3 --kinds "$KINDS" > "$R/gpurun_out/pmc_dw_${TAG}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmc_dw_${TAG}_$i.log"; exit 3; }
done
echo ok
