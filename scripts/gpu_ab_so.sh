#!/bin/bash
# Same-box A/B of the working tree ("new") against ab/base/ ("base": a git revision's package,
# bench.py and .so, prepared on the CPU host by scripts/ab_base.sh); interleaved bench runs.
# AB_TESTS: pytest selection run on the new build first; AB_ARGS: bench.py args.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abso && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/abso
PKG=pg---diploma-project---distributed-ai-model-training-using-mpi-and-accelerated-gpu-_amd
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
fi
rm -rf /tmp/abbase && cp -r ab/base /tmp/abbase || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py $AB_ARGS > $O/new_$i.json 2> $O/new.err || { tail -20 $O/new.err; exit 1; }
  (cd /tmp/abbase && PGDIST_AUTOBUILD=0 timeout -k 10 200 python -u bench.py $AB_ARGS > $O/base_$i.json 2> $O/base.err) || { tail -20 $O/base.err; exit 1; }
  python -c "import json; n=json.load(open('$O/new_$i.json'))['ms_per_step']; b=json.load(open('$O/base_$i.json'))['ms_per_step']; print('new', n, 'base', b)"
done
