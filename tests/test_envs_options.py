"""Env discovery fallbacks (``ddlb/envs.py``), option schema and registry aliases."""

import os

import pytest

from ddlb_amd import envs
from ddlb_amd.utils.options import EnvVarGuard, OptionsManager


def test_env_fallback_chain(monkeypatch):
    for k in ("OMPI_COMM_WORLD_RANK", "SLURM_PROCID", "PMI_RANK", "RANK", "OMPI_COMM_WORLD_SIZE",
              "SLURM_NTASKS", "PMI_SIZE", "WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK",
              "SLURM_LOCALID", "LOCAL_RANK", "DDLB_MASTER_PORT", "MASTER_PORT",
              "LOCAL_WORLD_SIZE", "TORCHELASTIC_RUN_ID"):
        monkeypatch.delenv(k, raising=False)
    assert envs.get_rank() == 0 and envs.get_world_size() == 1 and envs.get_local_rank() == 0
    monkeypatch.setenv("RANK", "3")
    assert envs.get_rank() == 3
    monkeypatch.setenv("PMI_RANK", "2")
    assert envs.get_rank() == 2
    monkeypatch.setenv("SLURM_PROCID", "1")
    assert envs.get_rank() == 1
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "5")
    assert envs.get_rank() == 5
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert envs.get_world_size() == 8
    assert envs.get_master_port() == 12345
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert envs.get_master_port() == 29501  # torchrun's agent owns MASTER_PORT
    monkeypatch.setenv("DDLB_MASTER_PORT", "4000")
    assert envs.get_master_port() == 4000


def test_options_manager():
    om = OptionsManager({"backend": "nccl", "s": 8, "flag": False},
                        {"backend": ["nccl", "rccl"], "s": (1, 64), "flag": [True, False]},
                        aliases={"backend": {"cuda": "rccl"}})
    om.parse({"implementation": "x", "backend": "cuda", "s": 4.0})
    assert om["backend"] == "rccl" and om["s"] == 4 and isinstance(om["s"], int)
    with pytest.raises(ValueError):
        OptionsManager({"a": 1}).parse({"b": 2})
    with pytest.raises(ValueError):
        OptionsManager({"s": 8}, {"s": (1, 64)}).parse({"s": 2.5})
    with pytest.raises(ValueError):
        OptionsManager({"s": 8}, {"s": (1, 64)}).parse({"s": 100})
    with pytest.raises(ValueError):
        OptionsManager({"b": "x"}, {"b": ["x", "y"]}).parse({"b": "z"})


def test_env_var_guard(monkeypatch):
    monkeypatch.setenv("DDLB_T1", "old")
    monkeypatch.delenv("DDLB_T2", raising=False)
    with EnvVarGuard({"DDLB_T1": "new", "DDLB_T2": "x"}):
        assert os.environ["DDLB_T1"] == "new" and os.environ["DDLB_T2"] == "x"
    assert os.environ["DDLB_T1"] == "old" and "DDLB_T2" not in os.environ


def test_registry_aliases():
    from ddlb_amd.primitives.registry import implementations, resolve

    cls, opts, note = resolve("tp_columnwise", "fuser", {"algorithm": "coll_pipeline", "s": 2,
                                                         "backend": "nccl", "bogus": 1})
    assert cls.__name__ == "NativeTPColumnwise" and "bogus" not in opts and opts["s"] == 2
    cls, opts, _ = resolve("tp_columnwise", "transformer_engine", {})
    assert opts["algorithm"] == "p2p_pipeline"
    cls, opts, _ = resolve("tp_rowwise", "jax", {})
    assert cls.__name__ == "NativeTPRowwise" and opts["algorithm"] == "default"
    assert "compute_only" in implementations("tp_rowwise")
    with pytest.raises(ValueError):
        resolve("tp_rowwise", "nope", {})


def test_ucc_backends_rejected():
    from ddlb_amd.primitives.backends import BackendUnavailable
    from ddlb_amd.primitives.native_common import COMMON_DEFAULTS, algo_config
    from ddlb_amd.utils.options import OptionsManager
    from ddlb_amd.primitives.native_common import COMMON_ALLOWED, COMMON_ALIASES

    om = OptionsManager(COMMON_DEFAULTS, COMMON_ALLOWED, COMMON_ALIASES)
    om.parse({"backend": "ucc/tl/nccl"})
    with pytest.raises(BackendUnavailable):
        algo_config(om)
    om = OptionsManager(COMMON_DEFAULTS, COMMON_ALLOWED, COMMON_ALIASES)
    om.parse({"backend": "cuda", "multicast_protocol": "multimem"})
    cfg = algo_config(om)
    assert cfg.backend == "ipc" and cfg.protocol == "kernel"


def _node_check_worker(rank, world, port, q, hosts):
    import os
    import socket

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    from ddlb_amd.parallel.context import check_single_node

    socket.gethostname = lambda: hosts[rank]  # this rank "runs" on hosts[rank]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        check_single_node(world)
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("hosts", [("a", "a"), ("a", "b")])
def test_ipc_single_node_check(hosts):
    """backend=ipc plans refuse a job that spans several hosts (HIP IPC / xGMI is per node)."""
    import multiprocessing as mp

    from conftest import free_port

    ctx = mp.get_context("spawn")
    q, port = ctx.Queue(), free_port()
    procs = [ctx.Process(target=_node_check_worker, args=(r, 2, port, q, hosts)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    if hosts[0] == hosts[1]:
        assert got == {0: "ok", 1: "ok"}
    else:
        assert all("one node" in v and "backend=rccl" in v for v in got.values()), got
