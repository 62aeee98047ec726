"""Rank / world / rendezvous discovery from the launcher environment.

Parity: ``ddlb/envs.py:12-82`` reads OpenMPI -> SLURM -> PMI variables with fallbacks.
We keep those chains and additionally read the variables torchrun exports
(``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR``,
``MASTER_PORT``), because on the MI355X boxes torchrun (not mpirun) is the launcher.

Nothing in this module touches the GPU: the parent process of the benchmark runner
uses it to decide rank-0 behaviour before any HIP context exists.
"""

from __future__ import annotations

import os
from typing import Optional, Sequence


def get_env(key: str, default: Optional[str] = None,
            fallback_keys: Optional[Sequence[str]] = None) -> str:
    """Return the first set variable among ``key`` and ``fallback_keys``, else ``default``."""
    for k in (key, *(fallback_keys or ())):
        v = os.getenv(k)
        if v is not None and v != "":
            return v
    return default if default is not None else ""


def get_rank() -> int:
    """Global rank: OMPI -> SLURM -> PMI -> torchrun -> 0."""
    return int(get_env("OMPI_COMM_WORLD_RANK", "0", ["SLURM_PROCID", "PMI_RANK", "RANK"]))


def get_local_rank() -> int:
    """Node-local rank: OMPI -> SLURM -> torchrun -> 0."""
    return int(get_env("OMPI_COMM_WORLD_LOCAL_RANK", "0", ["SLURM_LOCALID", "LOCAL_RANK"]))


def get_world_size() -> int:
    """World size: OMPI -> SLURM -> PMI -> torchrun -> 1."""
    return int(get_env("OMPI_COMM_WORLD_SIZE", "1", ["SLURM_NTASKS", "PMI_SIZE", "WORLD_SIZE"]))


def get_local_size() -> int:
    """Processes on this node: OMPI -> SLURM -> torchrun -> 1."""
    return int(get_env("OMPI_COMM_WORLD_LOCAL_SIZE", "1",
                       ["SLURM_NTASKS_PER_NODE", "LOCAL_WORLD_SIZE"]))


def get_master_addr() -> str:
    """Rendezvous host. 127.0.0.1 (not ``localhost``): container hostnames may not resolve."""
    return get_env("DDLB_MASTER_ADDR", "127.0.0.1", ["MASTER_ADDR"])


def under_torchrun() -> bool:
    """True when launched by torch.distributed.run (its agent owns MASTER_PORT)."""
    return "TORCHELASTIC_RUN_ID" in os.environ or (
        "MASTER_PORT" in os.environ and "LOCAL_WORLD_SIZE" in os.environ)


def get_master_port() -> int:
    """Base rendezvous port for the per-child process groups.

    ``DDLB_MASTER_PORT`` wins (reference default 12345). Under torchrun the agent already
    listens on ``MASTER_PORT``, so children use the ports just above it.
    """
    explicit = os.getenv("DDLB_MASTER_PORT")
    if explicit:
        return int(explicit)
    if under_torchrun():
        return int(os.environ["MASTER_PORT"]) + 1
    return 12345


def get_jax_coord_addr() -> str:
    """Kept for configuration parity (``ddlb/envs.py:80-82``); JAX is not a backend here."""
    return get_env("JAX_COORD_ADDR", "127.0.0.1:12355")
