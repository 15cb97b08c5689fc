#!/bin/bash
# Round 4: full GPU test suite + smoke on the current tree
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/suite && export TMPDIR=/tmp
O=gpurun_out/suite
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
