#!/bin/bash
# Dense-conv kernel probe: per-layer timings (scripts/conv_bench.py) and one counter pass per
# kernel family on a few compute-bound layers ($1: tag, $2: conv_bench kinds)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-base}; KINDS=${2:-fwd,dgradm,wgradma,wgrad}
O=gpurun_out/conv_$TAG; mkdir -p $O
timeout -k 10 300 python -u scripts/conv_bench.py --kinds $KINDS --reps 9 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
cat $O/bench.txt
if [ -n "$PMC" ]; then
  C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc" -o run -- \
    python3 "$GRAFT_REPO_ROOT/scripts/conv_bench.py" --kinds $KINDS --reps 2 --only l3.c2 > "$GRAFT_REPO_ROOT/$O/pmc.log" 2>&1 \
    || { tail -5 "$GRAFT_REPO_ROOT/$O/pmc.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT" && python3 scripts/pmc_table.py $O/pmc > $O/pmc_table.txt 2>&1; cat $O/pmc_table.txt | tail -30
fi
