#!/bin/bash
# Round 5: the whole GPU suite (one process) and the smoke entry point
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5full && export TMPDIR=/tmp
O=gpurun_out/r5full
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; exit $rc
