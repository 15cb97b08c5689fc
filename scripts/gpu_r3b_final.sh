#!/bin/bash
# checkpoint: full GPU suite + smoke, benches, ResNet-50 roofline + MobileNetV2 roofline
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
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
for cfg in "PGDIST_PW_WIDE_FWD=2" "PGDIST_PW_WIDE_FWD=1" "PGDIST_PW_WIDE_FWD=2" "PGDIST_PW_WIDE_FWD=1"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/fin_w.json 2> $O/fin_w.err || { tail -20 $O/fin_w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/fin_w.json')); print('$cfg', d['ms_per_step'])"
done
timeout -k 10 400 python -u scripts/roofline.py --model resnet50 --out $O/roofline_rn_fin.txt > $O/roofline_rn_fin.log 2>&1 && tail -22 $O/roofline_rn_fin.txt
timeout -k 10 400 python -u scripts/roofline.py --out $O/roofline_mb_fin.txt > $O/roofline_mb_fin.log 2>&1 && tail -24 $O/roofline_mb_fin.txt
