cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
PGDIST_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/b2.json 2> gpurun_out/b2.err || { tail -30 gpurun_out/b2.err; exit 3; }
cat gpurun_out/b2.json
