#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-pf}
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_trainer.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 50 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('prefetch', d['ms_per_step'], d['value'])"
PGDIST_AUG_PREFETCH=0 timeout -k 10 300 python bench.py --steps 50 > gpurun_out/bench_${TAG}0.json 2> gpurun_out/bench_${TAG}0.err || { tail gpurun_out/bench_${TAG}0.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}0.json'));print('no prefetch', d['ms_per_step'], d['value'])"
done
