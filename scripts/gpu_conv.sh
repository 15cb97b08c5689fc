#!/bin/bash
# Dense-conv kernel study on one GPU: isolated per-layer timing (scripts/conv_bench.py), then
# two PMC passes (kernel-trace only) over a few layers.  ONLY / KINDS select the PMC layers.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/conv && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 240 python scripts/conv_bench.py ${BENCH_ARGS:-} > gpurun_out/conv/bench.txt 2>&1 || { tail -20 gpurun_out/conv/bench.txt; exit 3; }
cat gpurun_out/conv/bench.txt
[ -n "$NO_PMC" ] && exit 0
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16"; do
  i=$((i+1))
  rm -rf "$R/gpurun_out/conv/p$i"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/conv/p$i" -o run -- python3 "$R/scripts/conv_bench.py" --reps 3 --only "${ONLY:-l3.c2}" --kinds "${KINDS:-fwd,fwdbn,dgrad}" > "$R/gpurun_out/conv/p$i.log" 2>&1)
  rc=$?; echo "pmc pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/conv/p$i.log"; exit $rc; }
done
python3 scripts/pmc_table.py gpurun_out/conv/p1 gpurun_out/conv/p2 --filter conv_ 2>&1 | tee gpurun_out/conv/pmc.txt | head -40
exit 0
