#!/bin/bash
# HIP API + kernel trace of the default bench (host-side submission timing)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; T=${1:-hip}
rm -rf gpurun_out/prof_$T
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d "$R/gpurun_out/prof_$T" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_$T.log" 2>&1) || exit 6
tail -1 gpurun_out/prof_$T.log; ls gpurun_out/prof_$T
