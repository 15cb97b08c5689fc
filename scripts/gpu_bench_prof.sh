#!/bin/bash
# Default bench (JSON line) + rocprofv3 kernel trace of the MobileNetV2 step; $1 = tag.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; TAG=${1:-cur}
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 4; }
cat gpurun_out/bench_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 3; }
echo prof ok
