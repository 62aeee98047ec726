"""Option schema shared by the native TP-Columnwise / TP-Rowwise implementations.

Keeps the reference ``fuser`` option names (``ddlb/primitives/TPColumnwise/fuser.py:160-178``,
``TPRowwise/fuser.py:182-198``) so reference JSON configs run unchanged:

=================================  ===============================================================
option                             meaning here
=================================  ===============================================================
backend                            ``rccl`` (alias ``nccl``) RCCL collectives on our own comm and
                                   streams; ``ipc`` (alias ``cuda``) HIP IPC symmetric memory over
                                   xGMI. ``ucc*`` -> explicit error.
algorithm                          ``default`` | ``coll_pipeline`` | ``p2p_pipeline``
s                                  coll_pipeline stages (>= 1)
offset_stream_indexing_by_rank     ring order: step j works on shard (r+j)%d
multicast_protocol                 ipc data movement: ``memcpy`` (copy engines, one queue per
                                   peer; = ``default``), ``batch_memcpy`` (all peers on one queue),
                                   ``kernel`` (CU copy kernel; ``multimem`` maps here: MI355X has
                                   no NVLS multicast)
inter_stream_synchronization       serialise the per-peer transfers
=================================  ===============================================================

Native-only: ``signal`` (``stream`` = hipStreamWrite/WaitValue32 memops, ``kernel`` = tiny spin
kernels), ``tile`` (GEMM tile or ``auto``), ``gemm_mode`` (``auto`` | ``mx`` for block-scaled fp8 |
``generic``; every mode is one of our MFMA kernels: hipBLASLt stays the ``pytorch`` slot's baseline),
``copy_blocks`` (CU budget of the kernel protocol), ``copy_streams`` (memcpy pulls: copy streams,
i.e. copy engines, per peer — a hedge for links faster than one engine), ``fused`` (p2p / coll: one
arrival-flag-gated GEMM; ``reserve_cus`` = CUs its persistent form leaves free for the
kernels that set the flags), ``graph`` (capture the plan once and replay it as one hipGraph launch;
signal plans read a device-side run counter; not for plans with RCCL calls, copy-engine-fed
flag-gated GEMMs or a CU split; ``auto``, the default = whenever capturable, the plan has more than
a few ops and the process has >= 4 HW queues), ``comm_cus`` (CU budget of the communication: the
side streams run on that many CUs via ``hipExtStreamCreateWithCUMask``, the GEMMs on the rest; 0 =
unmasked), ``register`` (RCCL buffers allocated with ``ncclMemAlloc`` and registered with
``ncclCommRegister`` for zero-copy transfers), ``trace`` (a roctx range per plan op, e.g.
``gemm s3`` / ``copy p2 b1``, for ``rocprofv3 --marker-trace --kernel-rename``; also
``DDLB_PLAN_TRACE=1``), ``direction`` (columnwise ipc: ``pull`` peers' shards, or
``push`` my shard into every peer's gather buffer with posted xGMI writes), ``ag_mode`` (the in-kernel
all-gather's copy variant, csrc/gemm/gemm.h ``AgMode`` bits: 1 plain stores + release fence instead
of write-through stores, 2 agent-scope acquire in the gated tiles, 4 16 loads in flight per lane,
8 more copy workgroups while the GEMM's tile rounds stay the same, 16 the launch waits for the
peers' ACKs itself; default 30).
"""

from __future__ import annotations

from ddlb_amd.parallel.algorithms import AlgoConfig
from ddlb_amd.parallel.plan import SIG_KERNEL, SIG_STREAM
from ddlb_amd.primitives.backends import UCC_BACKENDS, BackendUnavailable

COMMON_DEFAULTS = {
    "backend": "rccl",
    "algorithm": "default",
    "s": 8,
    "offset_stream_indexing_by_rank": True,
    "multicast_protocol": "memcpy",
    "inter_stream_synchronization": False,
    "signal": "stream",
    "tile": "auto",
    "gemm_mode": "auto",
    "copy_blocks": 64,
    "copy_streams": 1,
    "fused": False,
    "reserve_cus": 32,
    "graph": "auto",
    "direction": "pull",
    "ag_mode": 30,
    "comm_cus": 0,
    "register": False,
    "trace": False,
}
COMMON_ALLOWED = {
    "backend": ["rccl", "ipc", *UCC_BACKENDS],
    "algorithm": ["default", "coll_pipeline", "p2p_pipeline", "direct"],
    "s": (1, 1 << 20),
    "offset_stream_indexing_by_rank": [True, False],
    "multicast_protocol": ["memcpy", "batch_memcpy", "kernel"],
    "inter_stream_synchronization": [True, False],
    "signal": ["stream", "kernel"],
    "tile": ["auto", "256x256", "256x128", "128x256", "128x128", "256x256w4", "256x128w4",
             "i256", "i128", "i256w4", "t8", "pt8", "t4", "pt4"],
    "gemm_mode": ["auto", "mx", "generic"],
    "copy_blocks": (1, 4096),
    "copy_streams": (1, 4),
    "fused": [True, False],
    "reserve_cus": (0, 1024),
    "graph": [True, False, "auto"],
    "direction": ["pull", "push"],
    "ag_mode": (0, 31),
    "comm_cus": (0, 1024),
    "register": [True, False],
    "trace": [True, False],
}
COMMON_ALIASES = {
    "backend": {"nccl": "rccl", "cuda": "ipc"},
    "multicast_protocol": {"default": "memcpy", "multimem": "kernel"},
}

from ddlb_amd.ops.gemm import TILES as TILE_CODE  # noqa: E402  (one table: csrc/gemm/gemm.h)
MODE_CODE = {"auto": 0, "generic": 1, "mx": 2}


def algo_config(options, order: str = "AG_before") -> AlgoConfig:
    backend = options["backend"]
    if backend in UCC_BACKENDS:
        raise BackendUnavailable(
            f"backend '{backend}' needs UCC/UCX, which the MI355X stack does not ship; use "
            "backend=rccl (alias nccl) or backend=ipc (alias cuda)")
    if (options["fused"] and options["multicast_protocol"] == "kernel"
            and options["algorithm"] != "coll_pipeline"):
        raise ValueError("fused=True with CU copies (multicast_protocol=kernel) is the in-kernel "
                         "all-gather of algorithm=coll_pipeline; p2p fused needs copy-engine "
                         "transfers (memcpy | batch_memcpy)")
    return AlgoConfig(
        algorithm=options["algorithm"], backend=backend, order=order, s=int(options["s"]),
        ring=bool(options["offset_stream_indexing_by_rank"]),
        protocol=options["multicast_protocol"],
        inter_stream_sync=bool(options["inter_stream_synchronization"]),
        signal=SIG_STREAM if options["signal"] == "stream" else SIG_KERNEL,
        tile=TILE_CODE[options["tile"]], mode=MODE_CODE[options["gemm_mode"]],
        copy_blocks=int(options["copy_blocks"]), fused=bool(options["fused"]),
        reserve_cus=int(options.get("reserve_cus", 32)),
        copy_streams=int(options.get("copy_streams", 1)),
        direction=options.get("direction", "pull"), ag_mode=int(options.get("ag_mode", 30)),
        comm_cus=int(options.get("comm_cus", 0)), register=bool(options.get("register", False)))


def share_cus(cfg: AlgoConfig, communicator) -> AlgoConfig:
    """Ranks sharing one GPU (rehearsals, tests): a flag-gated persistent GEMM must not take the
    CUs the co-resident ranks' kernels need to set its flags, so each rank's gated launch is held
    to its share of the device."""
    import dataclasses

    import torch

    rpd = getattr(communicator, "ranks_per_device", 1)
    if rpd <= 1 or not cfg.fused:
        return cfg
    cus = torch.cuda.get_device_properties(communicator.device).multi_processor_count
    spare = cus - cus // rpd
    return dataclasses.replace(cfg, reserve_cus=max(cfg.reserve_cus, spare + 32),
                               ag_reserve=max(cfg.ag_reserve, spare + 8))


def dtype_codes(dtype_name: str):
    from ddlb_amd.parallel.plan import NAME_DT, DT_BF16, DT_FP8

    din = NAME_DT[dtype_name]
    dout = DT_BF16 if din == DT_FP8 else din
    return din, dout


GRAPH_MIN_OPS = 4  # graph=auto: plans this long (host-issued signals / copies per run) replay


def maybe_enable_graph(bound, option) -> bool:
    """Apply the ``graph`` option to a bound plan; returns whether graph replay is on. ``auto``
    replays plans whose per-run host work the graph removes (>= GRAPH_MIN_OPS ops); a
    one-GEMM plan (world 1) stays a plain launch: a replay would add the run-counter kernel."""
    if option is True or option == "true":
        bound.enable_graph(True)
        return True
    from ddlb_amd.parallel.context import graph_replay_supported

    if (option == "auto" and len(bound.plan.ops) >= GRAPH_MIN_OPS
            and bound.ex.graph_capturable() and graph_replay_supported()):
        bound.enable_graph(True)
        return True
    return False
