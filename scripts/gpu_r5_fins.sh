#!/bin/bash
# Round 5: side-stream BN finalizes deferred to the bucket points (lazy coefficients in the
# weight-gradient prologues) -- numerics, then bench A/B on one box
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5fin && export TMPDIR=/tmp
O=gpurun_out/r5fin
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_executor_teacher_forced_gpu.py tests/test_ddp_gpu.py tests/test_bn_lazy_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
cat > $O/ab.py <<'PY'
import sys, runpy
from pgdist.engine.executor import MobileNetV2Executor
MobileNetV2Executor.DEFER_SIDE_FINS = sys.argv.pop(1) == "1"
sys.argv[0] = "bench.py"
runpy.run_path("bench.py", run_name="__main__")
PY
for i in 1 2 3; do
  for m in 1 0; do
    PYTHONPATH=. timeout -k 10 200 python -u $O/ab.py $m > $O/bench_${m}_$i.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  done
  python -c "import json; r={m: json.load(open('$O/bench_'+m+'_$i.json'))['ms_per_step'] for m in ('1','0')}; print('deferred fins', r['1'], 'per-group fins', r['0'])"
done
