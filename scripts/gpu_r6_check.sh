#!/bin/bash
# Round 6 check: full GPU suite (one pytest process), smoke, one default bench run
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${T:-} > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
