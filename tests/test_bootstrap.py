"""Rank discovery (mpirun / SLURM / torchrun env) — multi-node correct, unlike the reference's
hard-coded MASTER_ADDR=localhost (cifar10_mpi_mobilenet_224.py:29)."""
from pgdist.parallel.bootstrap import discover, _first_slurm_host


def test_single_process_default():
    i = discover({})
    assert (i.rank, i.world_size, i.local_rank, i.is_distributed) == (0, 1, 0, False)


def test_torchrun_env():
    i = discover({"RANK": "5", "WORLD_SIZE": "16", "LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "8",
                  "MASTER_ADDR": "10.0.0.2", "MASTER_PORT": "1234"})
    assert (i.rank, i.world_size, i.local_rank, i.master_addr, i.master_port) == (5, 16, 1, "10.0.0.2", 1234)
    assert i.source == "env"


def test_openmpi_env():
    i = discover({"OMPI_COMM_WORLD_RANK": "3", "OMPI_COMM_WORLD_SIZE": "4", "OMPI_COMM_WORLD_LOCAL_RANK": "1",
                  "OMPI_COMM_WORLD_LOCAL_SIZE": "2"})
    assert (i.rank, i.world_size, i.local_rank, i.local_world_size, i.source) == (3, 4, 1, 2, "openmpi")


def test_slurm_env_multinode():
    i = discover({"SLURM_PROCID": "9", "SLURM_NTASKS": "16", "SLURM_LOCALID": "1",
                  "SLURM_JOB_NODELIST": "gpu[008-009]", "SLURM_NTASKS_PER_NODE": "8(x2)"})
    assert (i.rank, i.world_size, i.local_rank, i.local_world_size) == (9, 16, 1, 8)
    assert i.master_addr == "gpu008"


def test_nodelist_parsing():
    assert _first_slurm_host("gpu[008-011,020]") == "gpu008"
    assert _first_slurm_host("cn1,cn2") == "cn1"
    assert _first_slurm_host("node17") == "node17"
