#!/bin/bash
# Round 4 checkpoint: full GPU suite + smoke, MobileNetV2 / ResNet-50 benches, bf16 vs fp8 bs512
# back to back, rocprofv3 kernel statistics of the headline bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4f && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; O=gpurun_out/r4f
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20; tail -2 $O/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
ab() {
  t=$1; b=$2
  timeout -k 10 200 python -u $b --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
[ -f ab/base/bench.py ] && [ -n "$PGDIST_AB" ] && for i in 1 2 3; do ab base ab/base/bench.py; ab new bench.py; done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/mnv2_$i.json 2> $O/mnv2.err || { tail -20 $O/mnv2.err; exit 1; }
  cat $O/mnv2_$i.json
done
timeout -k 10 250 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn50.json 2> $O/rn50.err || { tail -20 $O/rn50.err; exit 1; }
cat $O/rn50.json
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --batch-size 512 --steps 20 --warmup 5 > $O/bf16_512_$i.json 2> $O/b512.err || { tail -20 $O/b512.err; exit 1; }
  timeout -k 10 300 python -u bench.py --batch-size 512 --fp8 1 --steps 20 --warmup 5 > $O/fp8_512_$i.json 2> $O/f512.err || { tail -20 $O/f512.err; exit 1; }
  python -c "import json; a=json.load(open('$O/bf16_512_$i.json')); b=json.load(open('$O/fp8_512_$i.json')); print('bs512 bf16', a['ms_per_step'], 'fp8', b['ms_per_step'])"
done
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 > "$R/$O/prof.log" 2>&1) || exit 6
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python scripts/kstats_top.py $f > $O/kstats_top.txt && head -30 $O/kstats_top.txt
