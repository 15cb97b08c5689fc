#!/bin/bash
# Round 4: executor tests with the small-map block-output fusion on by default; per-kernel trace
# of the bench step (augment params / render split)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/augprof && export TMPDIR=/tmp
O=gpurun_out/augprof
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_executor_teacher_forced_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/pytest.log | head -30; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/bench.log 2>&1
rc=$?; tail -1 $GRAFT_REPO_ROOT/$O/bench.log; exit $rc
