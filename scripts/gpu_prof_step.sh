#!/bin/bash
# Kernel trace of the default bench step (PROF_TAG names the output directory).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; T=${PROF_TAG:-step}
rm -rf gpurun_out/prof_$T
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$T" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 $PROF_ARGS > "$R/gpurun_out/prof_$T.log" 2>&1) || exit 6
tail -1 gpurun_out/prof_$T.log
