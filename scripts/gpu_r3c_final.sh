#!/bin/bash
# end-of-session checkpoint: full GPU suite + smoke, MobileNetV2 / ResNet-50 benches, bf16 vs fp8 bs512 back to back
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do ab geom3 X=1; ab geom2 PGDIST_DW_GEOM=2; done
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > $O/fin_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/fin_tests.log | head -20; tail -2 $O/fin_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/fin_smoke.log 2>&1 || { tail -20 $O/fin_smoke.log; exit 1; }
tail -1 $O/fin_smoke.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/fin_mb.json 2> $O/fin_mb.err || { tail -20 $O/fin_mb.err; exit 1; }
  cat $O/fin_mb.json
  timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/fin_rn.json 2> $O/fin_rn.err || { tail -20 $O/fin_rn.err; exit 1; }
  cat $O/fin_rn.json
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --batch-size 512 --steps 20 --warmup 5 > $O/fin_bf16_512.json 2> $O/fin_b512.err || { tail -20 $O/fin_b512.err; exit 1; }
  cat $O/fin_bf16_512.json
  timeout -k 10 300 python -u bench.py --batch-size 512 --fp8 1 --steps 20 --warmup 5 > $O/fin_fp8_512.json 2> $O/fin_f512.err || { tail -20 $O/fin_f512.err; exit 1; }
  cat $O/fin_fp8_512.json
done
