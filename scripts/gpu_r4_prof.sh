#!/bin/bash
# Round 4: per-op roofline of the replayed MobileNetV2 step + kernel-trace timeline of the bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; O=gpurun_out/r4; T=${TAG:-r4}
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$T.txt > $O/roofline_$T.log 2>&1
rc=$?; tail -25 $O/roofline_$T.txt; [ $rc -eq 0 ] || { tail -20 $O/roofline_$T.log; exit $rc; }
rm -rf $O/prof_$T
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$T" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 3 > "$R/$O/prof_$T.log" 2>&1) || exit 6
f=$(find $O/prof_$T -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py $f > $O/timeline_$T.txt && head -70 $O/timeline_$T.txt
