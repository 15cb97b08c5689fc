"""bench.py driver contract on the CPU (gloo): one JSON line from rank 0 with the metric /
config BASELINE.json names, whole-job aggregate throughput, max-over-ranks timing, and the
torch.distributed.run launch (127.0.0.1 rendezvous) the driver uses for N > 1.  The GPU
numbers themselves are produced on the MI355X box; this checks the plumbing."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = json.load(open(os.path.join(ROOT, "BASELINE.json")))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(env_extra=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return env


def _run(cmd, env_extra=None):
    r = subprocess.run(cmd, cwd=ROOT, env=_env(env_extra), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _check(d, n, steps, warmup, batch):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == batch * n and d["config"]["parallelism"] == f"dp{n}"
    # whole-job aggregate: images/s = global batch * steps / elapsed
    assert abs(d["value"] - batch * n * 1e3 / d["ms_per_step"]) / d["value"] < 0.02


def test_bench_single_process_cpu():
    d = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--batch-size", "2", "--img-size", "32"])
    _check(d, 1, 2, 1, 2)
    assert d["config"]["model"] == "mobilenet_v2"


@pytest.mark.slow
def test_bench_two_ranks_torchrun_cpu():
    port = _free_port()
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "2",
              "--warmup", "1", "--batch-size", "2", "--img-size", "32"])
    _check(d, 2, 2, 1, 2)
    # data-parallel health fields of an N > 1 run
    assert d["comm_error"] == 0 and d["replicas_identical"] is True and "rccl_ranks" in d
    assert d["config"]["bn_broadcast"] is True


@pytest.mark.slow
def test_bench_self_launches_without_launcher_cpu():
    """`bench.py --gpus 2` with no launcher must start 2 ranks itself (never a silent 1-rank run)."""
    d = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch-size", "2",
              "--img-size", "32"])
    _check(d, 2, 2, 1, 2)
    assert d["replicas_identical"] is True and d["comm_error"] == 0


@pytest.mark.slow
def test_bench_rank_count_mismatch_fails_cpu():
    """A launcher that started a different number of ranks than --gpus is an error, not a result."""
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "3",
                        "--steps", "1", "--warmup", "0", "--batch-size", "2", "--img-size", "32"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "WORLD_SIZE=2" in r.stderr


def test_headline_metric_matches_baseline():
    """At the headline config (MobileNetV2, bs 128/GPU, bf16) the metric string is BASELINE.json's."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert BASE["metric"] in src
