#!/bin/bash
# sanity of the final tree: smoke, kernel / conv GPU tests, one bench of each model
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s_smoke.log 2>&1 || { tail -20 $O/s_smoke.log; exit 1; }
tail -1 $O/s_smoke.log | cut -c1-60
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_resnet_executor_gpu.py tests/test_executor_gpu.py > $O/s_tests.log 2>&1 || { grep -E "FAILED|Error" $O/s_tests.log | head -20; tail -3 $O/s_tests.log; exit 1; }
tail -1 $O/s_tests.log
timeout -k 10 200 python -u bench.py > $O/s_mb.json 2> $O/s_mb.err || { tail -20 $O/s_mb.err; exit 1; }
python -c "import json; d=json.load(open('$O/s_mb.json')); print('mb', d['ms_per_step'], d['value'])"
timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/s_rn.json 2> $O/s_rn.err || { tail -20 $O/s_rn.err; exit 1; }
python -c "import json; d=json.load(open('$O/s_rn.json')); print('rn', d['ms_per_step'], d['value'])"
