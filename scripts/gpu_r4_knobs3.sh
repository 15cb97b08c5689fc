#!/bin/bash
# Round 4: main-stream gaps before the expand dgrad (kernel trace: 35-100 us per step while the
# side-stream weight gradients hold every CU slot): side-grid caps, main-stream priority, CU mask
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4k3 && export TMPDIR=/tmp
O=gpurun_out/r4k3
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do
  ab default X=1
  ab pwwg_wgs256 PGDIST_PWWG_WGS=256
  ab pwwg_wgs384 PGDIST_PWWG_WGS=384
  ab main_prio PGDIST_MAIN_PRIO=1
  ab side_cus7_8 PGDIST_SIDE_CUS=7/8
  ab side_cus3_4 PGDIST_SIDE_CUS=3/4
  ab wred_wgs128 PGDIST_WRED_WGS=128
done
