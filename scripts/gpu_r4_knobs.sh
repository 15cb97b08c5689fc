#!/bin/bash
# Round 4: re-sweep of the side-stream / tile knobs after the pw_tile shape rule and the faster
# pw_wgrad (same box, 2 reps each, bench ms/step)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do
  ab default X=1
  ab pwwg_wgs512 PGDIST_PWWG_WGS=512
  ab pwwg_wgs2048 PGDIST_PWWG_WGS=2048
  ab pwwg_small128 PGDIST_PWWG_MINROWS_SMALL=128
  ab pwwg_small512 PGDIST_PWWG_MINROWS_SMALL=512
  ab side_batch2 PGDIST_SIDE_BATCH=2
  ab side_batch4 PGDIST_SIDE_BATCH=4
  ab tile_k64_128 PGDIST_TILE_K64=128
  ab wred_wgs128 PGDIST_WRED_WGS=128
  ab bn_rep4 PGDIST_BN_REP=4
done
