#!/bin/bash
# Round 4 PMC passes on the MobileNetV2 step (kernel-trace only, one counter group per run)
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r4pmc"; mkdir -p "$O"; rm -rf "$O"/p*
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$O/p$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 3 > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/p$i.log"; exit $rc; fi
done
cd "$R" && python scripts/pmc_r4.py gpurun_out/r4pmc > gpurun_out/r4pmc/summary.txt && head -60 gpurun_out/r4pmc/summary.txt
