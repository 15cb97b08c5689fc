#!/bin/bash
# Round 4: isolated augmentation kernels (params / render) under rocprofv3, composite vs exact
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/augk && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/augk
cd /tmp
timeout -k 10 120 python3 $GRAFT_REPO_ROOT/scripts/aug_bench.py > $O/wall.log 2>&1 && cat $O/wall.log &&
PGDIST_AUG_EXACT=1 timeout -k 10 120 python3 $GRAFT_REPO_ROOT/scripts/aug_bench.py > $O/wall_exact.log 2>&1 && cat $O/wall_exact.log &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/aug_bench.py > $O/prof.log 2>&1
