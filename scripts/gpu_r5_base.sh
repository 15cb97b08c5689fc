#!/bin/bash
# Round 5 baseline on a fresh box: smoke, two headline benches, per-op roofline of the step
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5b && export TMPDIR=/tmp
O=gpurun_out/r5b
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/mnv2_$i.json 2> $O/mnv2.err || { tail -20 $O/mnv2.err; exit 1; }
  cat $O/mnv2_$i.json
done
timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline.txt > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
tail -25 $O/roofline.txt
