#!/bin/bash
# Per-op isolated roofline of the working tree ("new") and of ab/base/ ("base", prepared by
# scripts/ab_base.sh) on the same box: gpurun_out/abroof/{new,base}.txt
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abroof && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/abroof
rm -rf /tmp/abbase && cp -r ab/base /tmp/abbase && mkdir -p /tmp/abbase/scripts && cp scripts/roofline.py /tmp/abbase/scripts/ || exit 1
timeout -k 10 300 python -u scripts/roofline.py ${ROOF_ARGS} --out $O/new.txt > $O/new.log 2>&1 || { tail -20 $O/new.log; exit 1; }
(cd /tmp/abbase && PGDIST_AUTOBUILD=0 timeout -k 10 300 python -u scripts/roofline.py ${ROOF_ARGS} --out $O/base.txt > $O/base.log 2>&1) || { tail -20 $O/base.log; exit 1; }
head -1 $O/new.txt; head -1 $O/base.txt
grep -E "^total" $O/new.txt $O/base.txt
