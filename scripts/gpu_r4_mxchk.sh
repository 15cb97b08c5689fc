#!/bin/bash
# Round 4: fp8 numerics / executor tests and smoke with the default PGDIST_F8_MX=2, bs512 pair
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/mxc && export TMPDIR=/tmp
O=gpurun_out/mxc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_fused_gpu.py tests/test_bn_lazy_gpu.py tests/test_executor_gpu.py -k "fp8 or f8" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  for v in bf16 fp8; do
    a="--batch-size 512 --steps 20 --warmup 5"; [ $v = fp8 ] && a="$a --fp8 1"
    timeout -k 10 300 python -u bench.py $a > $O/b_${v}_$i.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_$i.json')); print('bs512 $v', d['ms_per_step'], d['value'])"
  done
done
