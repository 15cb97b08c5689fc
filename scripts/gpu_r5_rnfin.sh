#!/bin/bash
# Round 5: ResNet-50 BN finalize fused into the producing convs (last-arriver tail) vs a
# finalize launch after every producer -- numerics, then bench A/B on one box
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5rn && export TMPDIR=/tmp
O=gpurun_out/r5rn
timeout -k 10 500 python -u -m pytest tests/test_resnet_executor_gpu.py tests/test_conv_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
cat > $O/ab.py <<'PY'
import sys, runpy
from pgdist.engine.resnet_executor import ResNet50Executor
ResNet50Executor.FUSED_FIN = sys.argv.pop(1) == "1"
sys.argv[0] = "bench.py"
runpy.run_path("bench.py", run_name="__main__")
PY
for i in 1 2; do
  for m in 1 0; do
    PYTHONPATH=. timeout -k 10 200 python -u $O/ab.py $m --model resnet50 --steps 20 --warmup 5 > $O/bench_${m}_$i.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  done
  python -c "import json; r={m: json.load(open('$O/bench_'+m+'_$i.json'))['ms_per_step'] for m in ('1','0')}; print('fused fin', r['1'], 'finalize launches', r['0'])"
done
