#!/bin/bash
# PMC counter passes (kernel-trace only; never combined with sys/runtime traces).
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
for set in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_ANY" "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python "$R/bench.py" --steps 2 --warmup 1 --graph 0 > "$R/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc/p$i.log"; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
