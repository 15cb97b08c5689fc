#!/bin/bash
# PMC counter passes (kernel-trace only; never combined with sys/runtime traces).
# FETCH_SIZE must run alone: with WRITE_SIZE/TCC counters in the same pass the
# request exceeds the hardware counter budget and rocprofv3 hangs.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc"
rm -rf "$R/gpurun_out/pmc/p"*
i=0
for set in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc/p$i.log"; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
