#!/bin/bash
# A/B bench of env-var configurations: each argument is "ENV1=v ENV2=v ..." (or "-" for none);
# prints one "<config> <ms/step>" line per argument.  Extra bench args: $BENCH_ARGS.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=""
  env $cfg timeout -k 10 150 python bench.py --steps 40 --warmup 10 $BENCH_ARGS > gpurun_out/ab.json 2> gpurun_out/ab.err \
    || { echo "FAILED: $cfg"; tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('${cfg:-default}', d['ms_per_step'])"
done
