"""bench.py on the MI355X with 2 ranks sharing ONE GPU (gloo default group, native P2P
communicator over IPC-mapped staging, per-step BN-buffer broadcast): the data-parallel health
fields of the JSON line, and the failure path — a rank that skips one timed step's collectives
must make EVERY rank exit non-zero with a communicator error, within the
P2P timeout, instead of finishing a run on desynchronised gradients."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(extra_env, steps=4, timeout=240):
    env = dict(os.environ, PGDIST_DIST_BACKEND="gloo", PGDIST_COMM="p2p", PGDIST_COMM_TIMEOUT="4")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env.update(extra_env)
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", str(steps), "--warmup", "3", "--batch-size", "32"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines


def test_bench_two_ranks_one_gpu_health_fields():
    r, lines = _bench({})
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["comm_error"] == 0 and d["replicas_identical"] is True
    assert d["config"]["bn_broadcast"] is True
    assert d["config"]["allreduce"]["comm"] == "native"


def test_bench_rank_skipping_a_step_fails_every_rank():
    r, lines = _bench({"PGDIST_FAULT_SKIP_STEP": "1", "PGDIST_FAULT_RANK": "1"})
    assert r.returncode != 0, "a desynchronised data-parallel run must not exit 0"
    assert "data-parallel run FAILED" in r.stderr, r.stderr[-3000:]
    # both ranks report the failure (rank 0 timed out waiting; rank 1 learns it in the agreement)
    assert r.stderr.count("data-parallel run FAILED") == 2, r.stderr[-3000:]
    assert len(lines) == 1 and lines[0]["comm_error"] != 0
