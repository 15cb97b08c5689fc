#!/bin/bash
# Round 5, final code: the 8-rank one-GPU data-parallel rehearsal (gloo + native P2P), then
# bs512 bf16 vs fp8 (BASELINE config 5) back to back, two runs each.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5end && export TMPDIR=/tmp
O=gpurun_out/r5end
PGDIST_DIST_BACKEND=gloo PGDIST_COMM=p2p timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29573 bench.py --gpus 8 --steps 6 --warmup 3 \
  --batch-size 32 > $O/rehearsal8.json 2> $O/rehearsal8.err || { tail -20 $O/rehearsal8.err; exit 1; }
cat $O/rehearsal8.json
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --batch-size 512 --steps 20 --warmup 5 > $O/bs512_bf16_$i.json 2> $O/e.err || { tail -20 $O/e.err; exit 1; }
  timeout -k 10 300 python -u bench.py --batch-size 512 --steps 20 --warmup 5 --fp8 1 > $O/bs512_fp8_$i.json 2> $O/e.err || { tail -20 $O/e.err; exit 1; }
  python -c "import json; a=json.load(open('$O/bs512_bf16_$i.json')); b=json.load(open('$O/bs512_fp8_$i.json')); print('bf16', a['ms_per_step'], a['value'], 'fp8', b['ms_per_step'], b['value'])"
done
