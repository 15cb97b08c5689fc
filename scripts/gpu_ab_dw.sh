#!/bin/bash
# Isolated depthwise-kernel timings (scripts/dw_bench.py) of the working tree ("new") and of
# ab/base/ ("base", prepared by scripts/ab_base.sh) on one box, interleaved twice
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abdw && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/abdw
KINDS=${DW_KINDS:-dgrad,dgradw}
rm -rf /tmp/abbase && cp -r ab/base /tmp/abbase && mkdir -p /tmp/abbase/scripts && cp scripts/dw_bench.py /tmp/abbase/scripts/ || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u scripts/dw_bench.py --kinds $KINDS --reps 21 > $O/new_$i.txt 2>&1 || { tail -20 $O/new_$i.txt; exit 1; }
  (cd /tmp/abbase && PGDIST_AUTOBUILD=0 timeout -k 10 300 python -u scripts/dw_bench.py --kinds $KINDS --reps 21 > $O/base_$i.txt 2>&1) || { tail -20 $O/base_$i.txt; exit 1; }
done
for f in new_1 base_1 new_2 base_2; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
