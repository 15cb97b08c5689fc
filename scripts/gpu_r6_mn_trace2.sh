#!/bin/bash
# MobileNetV2 bs128 step kernel traces with the finalize launches (PGDIST_BN_LAZY=0) and lazy (default)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/mntrace && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/mntrace
for m in 0 1; do
  cd /tmp && PGDIST_BN_LAZY=$m timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $O/prof$m.log 2>&1 || { tail -20 $O/prof$m.log; exit 1; }
  cd $GRAFT_REPO_ROOT && python3 scripts/timeline.py $(find $O/prof$m -name "*kernel_trace.csv" | head -1) > $O/timeline_lazy$m.txt 2>&1
  head -50 $O/timeline_lazy$m.txt
done
