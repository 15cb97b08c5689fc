#!/bin/bash
# Round 4: kernel + executor GPU tests and smoke on the current defaults
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/chk && export TMPDIR=/tmp
O=gpurun_out/chk
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
