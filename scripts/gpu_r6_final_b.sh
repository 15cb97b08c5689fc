#!/bin/bash
# Round 6 final validation, part B: 20-epoch synthetic-hard gpu128 run + one planted-gradient-bug
# run (every depthwise weight gradient zeroed), the 8-rank one-GPU data-parallel rehearsal,
# bs512 bf16 vs fp8 back to back, ResNet-50 MFMA counter pass
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6final && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6final
timeout -k 10 300 python -u train.py --preset gpu128 --data synthetic-hard --epochs 20 --seed 1 \
  --save-path $O/best.pth > $O/e2e_hard_gpu128_20ep.log 2>&1 || { tail -10 $O/e2e_hard_gpu128_20ep.log; exit 1; }
grep -E "Best|Total" $O/e2e_hard_gpu128_20ep.log | tail -2
PGDIST_FAULT_ZERO_GRAD=@dw timeout -k 10 300 python -u train.py --preset gpu128 --data synthetic-hard --epochs 20 --seed 1 \
  --save-path $O/best_bug.pth > $O/e2e_hard_gpu128_20ep_bug_dw.log 2>&1 || { tail -10 $O/e2e_hard_gpu128_20ep_bug_dw.log; exit 1; }
grep -E "Best|Total" $O/e2e_hard_gpu128_20ep_bug_dw.log | tail -2
PGDIST_DIST_BACKEND=gloo PGDIST_COMM=p2p timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29583 bench.py --gpus 8 --steps 6 --warmup 3 \
  --batch-size 32 > $O/rehearsal8.out 2> $O/rehearsal8.err || { tail -20 $O/rehearsal8.err; exit 1; }
grep '^{' $O/rehearsal8.out | tail -1 > $O/rehearsal8.json; cat $O/rehearsal8.json
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --batch-size 512 --steps 20 --warmup 5 > $O/bs512_bf16_$i.json 2> $O/e.err || { tail -20 $O/e.err; exit 1; }
  timeout -k 10 300 python -u bench.py --batch-size 512 --steps 20 --warmup 5 --fp8 1 > $O/bs512_fp8_$i.json 2> $O/e.err || { tail -20 $O/e.err; exit 1; }
  python -c "import json; a=json.load(open('$O/bs512_bf16_$i.json')); b=json.load(open('$O/bs512_fp8_$i.json')); print('bf16', a['ms_per_step'], a['value'], 'fp8', b['ms_per_step'], b['value'])"
done
bash scripts/gpu_pmc_mfma.sh "resnet50_bs128:--model resnet50" "mnv2_bs128:--model mobilenet_v2"
