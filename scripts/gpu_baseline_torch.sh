#!/bin/bash
# Baseline: PyTorch/MIOpen path (channels_last bf16 autocast) on one MI355X.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 400 python bench.py --backend torch --steps 20 --warmup 10 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err &&
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_torch" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --backend torch --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_torch.log" 2>&1
