#!/bin/bash
# New GPU tests, then the multi-rank bench rehearsed with 2 ranks sharing one MI355X: gloo default
# group (RCCL refuses two ranks on one GPU), gradient buckets through the native P2P kernels.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_comm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit $rc
PGDIST_DIST_BACKEND=gloo PGDIST_COMM=p2p timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_2rank_p2p.json 2> gpurun_out/bench_2rank_p2p.err || { tail -20 gpurun_out/bench_2rank_p2p.err; exit 4; }
cat gpurun_out/bench_2rank_p2p.json
PGDIST_DIST_BACKEND=gloo PGDIST_COMM=c10d timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_2rank_c10d.json 2> gpurun_out/bench_2rank_c10d.err || { tail -20 gpurun_out/bench_2rank_c10d.err; exit 5; }
cat gpurun_out/bench_2rank_c10d.json
