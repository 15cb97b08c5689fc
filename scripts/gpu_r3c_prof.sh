#!/bin/bash
# rocprofv3 kernel statistics of the final tree (MobileNetV2 and ResNet-50 bs128 steps)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mb -o run -- python3 bench.py --steps 10 --warmup 5 > $O/prof_mb.log 2>&1 || { tail -20 $O/prof_mb.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn -o run -- python3 bench.py --model resnet50 --steps 10 --warmup 5 > $O/prof_rn.log 2>&1 || { tail -20 $O/prof_rn.log; exit 1; }
find $O/prof_mb $O/prof_rn -name "*kernel_stats.csv" | head
