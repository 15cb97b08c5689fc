#!/bin/bash
# ResNet-50 bs128 step kernel trace (rocprofv3 --kernel-trace) -> scripts/timeline.py summary
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rntrace && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/rntrace
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/timeline_rn50.txt 2>&1; head -60 $O/timeline_rn50.txt
