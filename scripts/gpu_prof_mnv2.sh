#!/bin/bash
# rocprofv3 kernel trace + stats of the MobileNetV2 bench step (eager, side stream on).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_mnv2" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_mnv2.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_mnv2.log"; exit 3; }
tail -1 "$R/gpurun_out/prof_mnv2.log"
find "$R/gpurun_out/prof_mnv2" -name "*.csv" | head
