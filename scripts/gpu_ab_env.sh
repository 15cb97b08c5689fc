#!/bin/bash
# Same-box A/B of environment knobs on one build: AB_VARS is a space-separated list of
# NAME=VALUE settings (several joined by "+"; "-" for the default), each one benched AB_REPS times, interleaved.
# AB_TESTS: pytest selection run first under every non-default setting; AB_ARGS: bench.py args.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abenv && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/abenv
if [ -n "$AB_TESTS" ]; then
  for v in $AB_VARS; do
    [ "$v" = "-" ] && continue
    env ${v//+/ } timeout -k 10 600 python -u -m pytest $AB_TESTS -x -q --timeout 300 --timeout-method thread \
      > $O/tests.log 2>&1
    rc=$?; echo "tests [$v]: $(grep -E 'passed|failed' $O/tests.log | tail -1)"; [ $rc -ne 0 ] && exit $rc
  done
fi
for i in $(seq 1 ${AB_REPS:-3}); do
  line="run $i:"
  for v in $AB_VARS; do
    tag=${v//[^A-Za-z0-9]/_}
    if [ "$v" = "-" ]; then
      timeout -k 10 200 python -u bench.py $AB_ARGS > $O/${tag}_$i.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    else
      env ${v//+/ } timeout -k 10 200 python -u bench.py $AB_ARGS > $O/${tag}_$i.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    fi
    ms=$(python -c "import json; print(json.load(open('$O/${tag}_$i.json'))['ms_per_step'])")
    line="$line  [$v] $ms"
  done
  echo "$line"
done
