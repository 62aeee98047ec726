"""Distributed-GEMM algorithms as plan builders (the native replacements of the nvFuser slots).

Reference semantics and where each is cited:

TP-Columnwise  (C[m,n] = AllGather_M(A_r[m/d,k]) @ B[k,n], rows rank-major)
  default        AG then GEMM                          ``TPColumnwise/fuser.py:16-57``
  coll_pipeline  s stages of (AG of m/(ds) rows from every rank || GEMM of the previous stage)
                                                        ``TPColumnwise/fuser.py:59-100``
  p2p_pipeline   d steps; step j computes shard (r+j)%d when offset_stream_indexing_by_rank
                                                        ``TPColumnwise/fuser.py:102-146``
  order=AG_after GEMM the local shard, all-gather C     ``fuser.py:200-201``
TP-Rowwise     (out_r[m/d,n] = ReduceScatter_M(A_r[m,k/d] @ B_r[k/d,n]))
  default        GEMM then RS                          ``TPRowwise/fuser.py:15-60``
  coll_pipeline  s stages of (GEMM of the d row blocks of stage j || RS of stage j-1). The native
                 layout keeps the canonical contiguous output block per rank (SURVEY.md §2.6
                 "Row coll_pipeline" native decision): stage j reads rows {r'*m/d + j*m/(sd) + i}
                 of A through the GEMM's grouped-row addressing — no permutation copy.
  p2p_pipeline   d steps; partial for destination (r+j)%d computed and shipped while the next
                 is computed; the destination sums d partials (f32) in one fused kernel.
                                                        ``TPRowwise/fuser.py:116-169``

Backends: ``rccl`` = RCCL collectives / send-recv on our own communicator and HIP streams;
``ipc`` = HIP IPC symmetric memory over xGMI, moved by the copy engines (SDMA, protocol
``memcpy``/``batch_memcpy``) or by CU copy kernels (``kernel``, the stand-in for NVLS
``multimem``), synchronised with cross-process flags (READY / ACK epochs).

Stream map: 0 = caller/compute, 1 = RCCL comm (high priority), 2.. = one copy stream per peer.

Enqueue order = intended time order. HIP multiplexes a process's streams onto a few hardware
queues (``GPU_MAX_HW_QUEUES``, 4 by default; a plan at d = 8 uses up to 9 streams). Kernels of
streams sharing a queue were measured to still overlap (profiles/r01/queue_blocking_check.txt),
but the builders emit ops stage by stage anyway — the copies of chunk j of every peer, then the
GEMM of stage j, then chunk j+1 — never all of one peer's chunks before the first GEMM: every
dependency then points backwards in enqueue order, which is what a fully in-order queue needs
(the world-4 GPU tests run with one queue per process) and what costs nothing otherwise. The
stream memops behind signal / wait are themselves rocclr blit kernels
(``__amd_rocclr_streamOpsWrite`` / ``streamOpsWait``, profiles/r02/sig9*).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

from ddlb_amd.parallel.plan import (COPY_ENGINE, COPY_KERNEL, DT_SIZE, DT_U8, OP_GEMM,
                                    SIG_IN_LAUNCH, SIG_KERNEL, SIG_STREAM, Plan, Ref)

S_MAIN, S_COMM = 0, 1
TILE_PT4 = 19  # csrc/gemm/gemm.h Tile::TILE_PT4 (the only kernel carrying in-kernel copies)
AG_WAIT_ACKS = 16  # csrc/gemm/gemm.h AgMode: the launch waits for the peers' ACKs itself


def _s_copy(i: int) -> int:
    return 2 + i


@dataclass
class AlgoConfig:
    algorithm: str = "default"          # default | coll_pipeline | p2p_pipeline
    backend: str = "rccl"               # rccl | ipc
    order: str = "AG_before"            # AG_before | AG_after (columnwise)
    s: int = 8                          # coll_pipeline stages
    ring: bool = True                   # offset_stream_indexing_by_rank
    protocol: str = "memcpy"            # memcpy | batch_memcpy | kernel   (ipc)
    inter_stream_sync: bool = False     # serialise the per-peer transfers
    signal: int = SIG_STREAM            # flag ops: stream memops (default) or kernels
    tile: int = 0                       # GEMM tile (0 = auto)
    mode: int = 0                       # GEMM mode (0 auto, 2 MX-fp8)
    copy_blocks: int = 64               # CU budget of the kernel copy protocol
    copy_streams: int = 1               # memcpy pulls: copy streams (copy engines) per peer
    fused: bool = False                 # columnwise p2p / coll: one flag-gated GEMM launch
    reserve_cus: int = 32               # fused: CUs the persistent gated GEMM leaves free
    ag_reserve: int = 0                 # in-kernel all-gather: CUs left free besides its copiers
    # in-kernel all-gather variant (csrc/gemm/gemm.h AgMode): 14 = write-through publication, 16
    # loads in flight per lane, agent-scope gate acquire (the fastest at world 1,
    # profiles/r02/s4/r2s4_2_agk_world1_modes.txt), copy workgroups grown while the GEMM's tile
    # rounds stay the same (flagship: 48 instead of 32 at no GEMM cost, r2s4_5_*); + 16: the
    # launch waits for the peers' ACKs itself (no wait kernel after it)
    ag_mode: int = 30
    act: int = 0                        # columnwise: fused GEMM epilogue activation (ACT_*)
    direction: str = "pull"             # columnwise ipc: pull peers' shards | push mine to peers
    # CU budget of the communication: side streams on comm_cus CUs
    # (hipExtStreamCreateWithCUMask), stream-0 GEMMs on the complement; 0 = unmasked
    comm_cus: int = 0
    register: bool = False              # RCCL buffers from ncclMemAlloc + ncclCommRegister
    # RCCL-fed fused GEMM: enqueue the gated GEMM BEFORE the stage collectives, so its own (never
    # gated) tiles start at once instead of after the host has enqueued every collective (RCCL
    # calls cost the host several us each); needs the GEMM and the comm stream on different
    # hardware queues (GPU_MAX_HW_QUEUES >= 2; the plan builder falls back otherwise)
    gemm_first: bool = True
    # RCCL-fed fused GEMM: raise a stage's arrival flags from a third stream behind an event
    # (True: the next collective never waits behind a signal kernel) or from the comm stream right
    # after the collective (False, the default: the event hand-off cost more than the signal
    # kernel in the queue, 0.19 vs 0.23 ms (s4) emulated at d = 8 with fast and with link-like
    # slow collectives, profiles/r04/r4_12_ab_*)
    sig_side: bool = False


@dataclass
class TensorLoc:
    buf: str
    off: int
    rows: int
    cols: int
    dtype: int


@dataclass
class PlanIO:
    a: TensorLoc
    b: TensorLoc
    out: TensorLoc


def _nstreams(d: int, per_peer: int = 1) -> int:
    return 2 + max(d - 1, 1) * max(per_peer, 1)


def _peer_order(rank: int, d: int, ring: bool) -> List[int]:
    """Order of the *other* ranks: (r+1)%d, (r+2)%d, ... with ring indexing, else ascending."""
    if ring:
        return [(rank + j) % d for j in range(1, d)]
    return [p for p in range(d) if p != rank]


def _shard_order(rank: int, d: int, ring: bool) -> List[int]:
    """Compute order of the d shards: own first (ring) or 0..d-1 (reference without offset)."""
    if ring:
        return [(rank + j) % d for j in range(d)]
    return list(range(d))


class _Flags:
    """Named slot table inside the symmetric ``flags`` buffer (uint32 words)."""

    def __init__(self, plan: Plan, d: int, s: int, symmetric: bool = True):
        self.d = d
        self.slots: Dict[str, Tuple[int, int]] = {}
        self.words = 0
        for name, count in (("READY", d), ("ACK", d), ("CHUNK", s * d), ("ACKS", s * d),
                            ("ARRIVE", s * d),  # ARRIVE[p * s + b]: block b of shard p landed
                            ("CNT", s * d + d)):  # in-kernel all-gather counters (monotonic)
            self.slots[name] = (self.words, count)
            self.words += count
        nbytes = max(256, ((self.words * 4 + 255) // 256) * 256)
        # local-only flags (RCCL-fed gated GEMMs: set by this rank's own signal kernels)
        plan.buffer("flags", nbytes, symmetric=symmetric, zero=True)

    def ref(self, name: str, idx: int, owner: Optional[int] = None) -> Ref:
        base, count = self.slots[name]
        if not 0 <= idx < count:
            raise IndexError(f"flag {name}[{idx}] out of range")
        return Ref("flags", 4 * (base + idx), owner)


def _finish(plan: Plan, cfg: AlgoConfig) -> None:
    """Record the data-plane settings the binder applies (CU split, RCCL registration) and size
    the compute-stream GEMMs to the CUs a split leaves them: a persistent GEMM's grid is one
    workgroup per CU, so on a masked stream it must not count the communication's CUs."""
    plan.meta.update(comm_cus=cfg.comm_cus, register=cfg.register)
    if cfg.comm_cus > 0:
        # every persistent launcher (pt4 plain / gated / in-kernel all-gather, pt8) sizes its
        # grid to num_cus - reserve_cus: on the masked compute stream no workgroup may wait for a
        # CU the communication holds
        for op in plan.ops:
            if op.kind == OP_GEMM and op.stream == S_MAIN:
                op.args["reserve_cus"] = max(op.args.get("reserve_cus", 0), cfg.comm_cus)


def _split_k(plan: Plan, M: int, N: int, K: int, ein: int, cfg: AlgoConfig) -> int:
    """K-slices for ONE full GEMM whose 256x256 grid would leave most of the 256 CUs idle (e.g.
    8192 x 1024 x 8192, BASELINE config #2: 128 tiles; ``ops.gemm.split_k_factor``): the
    persistent kernel runs every (slice, tile) pair in one launch (GemmArgs::ksplit) and a
    reduce op sums the partials. Auto tiles and no fused activation only. 1 = no split."""
    from ddlb_amd.ops.gemm import split_k_factor

    if cfg.tile != 0 or cfg.act:
        return 1
    return split_k_factor(M, N, K, ein)


def _full_gemm(plan: Plan, a_ref: Ref, Bt: Ref, c_ref: Ref, M: int, N: int, K: int, ein: int,
               eout: int, cfg: AlgoConfig, gdt: dict, tag: str = "KS") -> None:
    """C[M, N] = A[M, K] Bt^T on stream 0, K-split when :func:`_split_k` says so: ONE launch runs
    the S (slice, tile) pairs (slice s = K/S columns of A and Bt).

    Default: the launch writes S partials (output dtype) to a scratch buffer and a reduce op sums
    them in f32 into C (BASELINE config #2 shape: 0.1009 ms, r4_22). (A form that reduced inside
    the launch -- the last slice of each tile summing the others' f32 partials -- was measured
    slower, GEMM 0.1128 vs 0.1022 ms, profiles/r05/r5_19, and retired in round 6: every
    workgroup finishes its single tile together, so the partial stores, the arrival poll and the
    partial loads form one serial chain at the end of the kernel.)"""
    S = _split_k(plan, M, N, K, ein, cfg)
    if S == 1:
        plan.gemm(S_MAIN, a_ref, Bt, c_ref, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, **gdt)
        return
    part = plan.buffer(tag, S * M * N * eout)
    plan.gemm(S_MAIN, a_ref, Bt, part, M=M, N=N, K=K // S, lda=K, ldb=K, ldc=N, ksplit=S,
              **dict(gdt, tile=TILE_PT4))
    plan.reduce(S_MAIN, c_ref, [part + j * M * N * eout for j in range(S)], M * N, gdt["dout"])


# A flag-gated persistent GEMM fed by other kernels (RCCL, copy / signal kernels) must leave one CU
# free in EVERY shader array: the dispatcher places a kernel's workgroups on the shader arrays in
# turn and does not move one to another array when its array is full, so a single feeder
# workgroup assigned to an array whose every CU holds a spinning gated tile blocks the feeder,
# whatever the other arrays have free. MI355X: 32 arrays (4 per XCD) of 8 active CUs (KFD topology:
# array_count 32, cu_per_simd_array 9 of which 8 enabled); the gated grid is spread evenly (one
# workgroup per CU, round-robin), so a reserve of one CU per array (256 / 8 = 32) leaves every array
# a free CU. Measured (research/diag/diag_gate_placement.py, profiles/r05/r5_6_gate_placement.txt): grid
# 224 (reserve 32) ran with feeders of 32, 64 and 256 workgroups; 232 (reserve 24) blocked with 32
# or 256 and ran with 8; 240 (reserve 16) blocked with 64, ran with 16 -- exactly the hangs of
# profiles/r04/r4_32..r4_36. Smaller requests are raised to this floor.
CUS_PER_SHADER_ARRAY = 8


def min_gate_reserve(ncu: int = 0) -> int:
    """One free CU per shader array of the device (32 on a whole MI355X; a compute partition
    with fewer CUs has proportionally fewer arrays)."""
    from ddlb_amd.ops.gemm import device_cus

    return max(1, (ncu or device_cus()) // CUS_PER_SHADER_ARRAY)


MIN_GATE_RESERVE = 32  # min_gate_reserve() of a whole MI355X


def _gate_reserve(cfg: AlgoConfig) -> int:
    return max(cfg.reserve_cus, min_gate_reserve())


def _unique(events):
    """Events in first-seen order without repeats (a wait per distinct event is enough)."""
    seen: List[int] = []
    for e in events:
        if e not in seen:
            seen.append(e)
    return seen


def _chunks(flags: List[Ref], n: int = 16):
    for i in range(0, len(flags), n):
        yield flags[i:i + n]


def _signal(plan: Plan, stream: int, flags: List[Ref], cfg: AlgoConfig, delta: int = 0):
    for c in _chunks(flags):
        plan.signal(stream, c, method=cfg.signal, delta=delta)


def _wait(plan: Plan, stream: int, flags: List[Ref], cfg: AlgoConfig, delta: int = 0):
    for c in _chunks(flags):
        plan.wait_signal(stream, c, method=cfg.signal, delta=delta)


# =====================================================================================
#  TP-Columnwise
# =====================================================================================
def check_columnwise(d: int, m: int, n: int, k: int, cfg: AlgoConfig, ein: int = 2) -> None:
    if m % d:
        raise ValueError(f"m ({m}) must be divisible by world_size ({d})")
    if cfg.algorithm == "coll_pipeline" and m % (d * cfg.s):
        raise ValueError(f"m ({m}) must be divisible by s*world_size ({cfg.s}*{d}) for "
                         "coll_pipeline")
    if cfg.algorithm not in ("default", "coll_pipeline", "p2p_pipeline", "direct"):
        raise ValueError(f"unknown algorithm {cfg.algorithm}")
    if cfg.backend not in ("rccl", "ipc"):
        raise ValueError(f"unknown backend {cfg.backend}")
    if cfg.algorithm == "direct" and (cfg.backend != "ipc" or cfg.order != "AG_before"):
        raise ValueError("algorithm=direct reads peer shards over xGMI: backend=ipc, AG_before")
    if cfg.protocol not in ("memcpy", "batch_memcpy", "kernel"):
        raise ValueError(f"unknown protocol {cfg.protocol}")
    if cfg.direction not in ("pull", "push"):
        raise ValueError(f"unknown direction {cfg.direction}")
    if cfg.direction == "push" and (cfg.backend != "ipc" or cfg.order != "AG_before" or
                                    cfg.algorithm == "direct" or cfg.fused):
        raise ValueError("direction=push applies to backend=ipc, order=AG_before, "
                         "default / coll_pipeline / p2p_pipeline (not fused)")
    if cfg.fused and (cfg.order != "AG_before" or
                      cfg.algorithm not in ("p2p_pipeline", "coll_pipeline")):
        raise ValueError("fused=True (one arrival-flag-gated GEMM) applies to order=AG_before, "
                         "p2p_pipeline / coll_pipeline")
    if (cfg.fused and cfg.protocol == "kernel" and cfg.algorithm == "coll_pipeline" and d > 1
            and (m % 256 or n % 256 or k * ein % 256 or k * ein < 256 or cfg.act)):
        raise ValueError("the in-kernel all-gather (coll_pipeline, fused, kernel copies) runs on "
                         "the persistent 256x256 GEMM: m and n multiples of 256, k rows of an "
                         "even number of 128-byte K-tiles, no fused activation")
    if d > 17:
        raise ValueError("at most 17 ranks per node are supported by the flag/reduce ops")


def build_tp_columnwise(rank: int, d: int, m: int, n: int, k: int, din: int, dout: int,
                        cfg: AlgoConfig) -> Tuple[Plan, PlanIO]:
    plan, io = _build_tp_columnwise(rank, d, m, n, k, din, dout, cfg)
    _finish(plan, cfg)
    return plan, io


def _build_tp_columnwise(rank: int, d: int, m: int, n: int, k: int, din: int, dout: int,
                         cfg: AlgoConfig) -> Tuple[Plan, PlanIO]:
    check_columnwise(d, m, n, k, cfg, DT_SIZE[din])
    ein, eout = DT_SIZE[din], DT_SIZE[dout]
    ml = m // d
    ns = _nstreams(d, cfg.copy_streams)
    plan = Plan(rank, d, nstreams=ns, stream_priority=[0, 1] + [1] * (ns - 2))
    plan.meta.update(primitive="tp_columnwise", algorithm=cfg.algorithm, backend=cfg.backend,
                     order=cfg.order, copy_streams=cfg.copy_streams if cfg.protocol == "memcpy" else 1)
    Bt = plan.buffer("Bt", n * k * ein)
    A = (plan.buffer("A_full", m * k * ein, symmetric=(cfg.backend == "ipc"))
         if cfg.algorithm != "direct" else None)
    flags = (_Flags(plan, d, max(cfg.s, 1))
             if cfg.backend == "ipc" and d > 1 and cfg.algorithm != "direct" else None)
    gdt = dict(din=din, dout=dout, tile=cfg.tile, mode=cfg.mode, act=cfg.act)
    comm_dt = DT_U8 if ein == 1 else din   # fp8 moves as bytes

    def arow(r0: int) -> Ref:
        return A + r0 * k * ein

    if cfg.algorithm == "direct":
        return _col_direct(plan, rank, d, m, n, k, din, dout, ein, eout, cfg, gdt), \
            PlanIO(TensorLoc("A_own", 0, ml, k, din), TensorLoc("Bt", 0, n, k, din),
                   TensorLoc("C", 0, m, n, dout))

    if cfg.order == "AG_after":
        C = plan.buffer("C_full", m * n * eout, symmetric=(cfg.backend == "ipc"))
        io = PlanIO(TensorLoc("A_full", rank * ml * k * ein, ml, k, din),
                    TensorLoc("Bt", 0, n, k, din), TensorLoc("C_full", 0, m, n, dout))
        _col_ag_after(plan, rank, d, m, n, k, ein, eout, dout, cfg, A, Bt, C, flags, gdt)
        return plan, io

    C = plan.buffer("C", m * n * eout)
    io = PlanIO(TensorLoc("A_full", rank * ml * k * ein, ml, k, din),
                TensorLoc("Bt", 0, n, k, din), TensorLoc("C", 0, m, n, dout))

    def crow(r0: int) -> Ref:
        return C + r0 * n * eout

    def gemm(stream, a_ref, c_ref, M, **kw):
        plan.gemm(stream, a_ref, Bt, c_ref, M=M, N=n, K=k, lda=k, ldb=k, ldc=n, **gdt, **kw)

    def shard_gemm(p):  # shard p's rows on stream 0 (K-split when few tiles and long K)
        _full_gemm(plan, arow(p * ml), Bt, crow(p * ml), ml, n, k, ein, eout, cfg, gdt, tag="KSP")

    if d == 1:
        _full_gemm(plan, A, Bt, C, m, n, k, ein, eout, cfg, gdt)
        return plan, io

    alg, be = cfg.algorithm, cfg.backend
    if be == "ipc" and cfg.direction == "push":
        _col_push(plan, rank, d, ml, cfg, flags, arow, crow, gemm, k * ein)
        return plan, io
    if alg == "default" and be == "rccl":
        plan.allgather(S_MAIN, arow(rank * ml), A, ml * k, comm_dt)
        _full_gemm(plan, A, Bt, C, m, n, k, ein, eout, cfg, gdt)
    elif alg == "default" and be == "ipc":
        done = _ipc_pull_shards(plan, rank, d, cfg, flags, [(p, [(p * ml, ml)]) for p in
                                                             _peer_order(rank, d, cfg.ring)],
                                lambda r0: arow(r0), k * ein)
        for e in _unique(e for ev in done.values() for e in ev):
            plan.wait(S_MAIN, e)
        _full_gemm(plan, A, Bt, C, m, n, k, ein, eout, cfg, gdt)
        _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in range(d) if p != rank], cfg)
    elif alg == "coll_pipeline" and be == "rccl" and cfg.fused:
        _col_rccl_fused_coll(plan, rank, d, m, n, k, ein, cfg, A, Bt, C, comm_dt, gdt)
    elif alg == "p2p_pipeline" and be == "rccl" and cfg.fused:
        _col_rccl_fused_p2p(plan, rank, d, m, n, k, ein, cfg, A, Bt, C, comm_dt, gdt)
    elif alg == "coll_pipeline" and be == "rccl":
        rows = ml // cfg.s
        for j in range(cfg.s):
            stg = plan.buffer(f"STG{j}", d * rows * k * ein)
            plan.allgather(S_COMM, arow(rank * ml + j * rows), stg, rows * k, comm_dt)
            e = plan.event()
            plan.record(S_COMM, e)
            plan.wait(S_MAIN, e)
            gemm(S_MAIN, stg, crow(j * rows), d * rows, c_grp=rows, c_gstride=ml)
    elif alg == "coll_pipeline" and be == "ipc" and cfg.fused and cfg.protocol == "kernel":
        # In-kernel all-gather: ONE launch. Its first copy_blocks workgroups pull row block b
        # of every peer over xGMI (block-major, ring order) and set ARRIVE[p * s + b] when a
        # block has landed; the other workgroups run the persistent GEMM gated on those flags
        # (csrc/gemm/gemm_kernels.h ag_copy_role). No copy streams, no host op per block:
        # READY out, own blocks marked, one kernel, ACKs back.
        rows = ml // cfg.s
        _signal(plan, S_MAIN, [flags.ref("READY", rank, owner=p) for p in range(d) if p != rank],
                cfg)
        _signal(plan, S_MAIN, [flags.ref("ARRIVE", rank * cfg.s + j) for j in range(cfg.s)], cfg)
        seg = rows * k * ein
        in_launch = bool(cfg.ag_mode & AG_WAIT_ACKS)
        ag = dict(ctas=cfg.copy_blocks, parts=max(1, min(seg // (256 << 10), 1024)), rank=rank,
                  src=[A.at(p) for p in range(d)],
                  ack=[flags.ref("ACK", rank, owner=p) for p in range(d)],
                  ready=flags.ref("READY", 0), count=flags.ref("CNT", 0), mode=cfg.ag_mode,
                  wait_acks=[flags.ref("ACK", p) for p in range(d)] if in_launch else None)
        gdt_ag = dict(gdt, tile=TILE_PT4)
        plan.gemm(S_MAIN, A, Bt, C, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, **gdt_ag,
                  flags=flags.ref("ARRIVE", 0), flag_rows=rows, nshards=d * cfg.s, nsub=cfg.s,
                  first_shard=rank, tile_order=1, reserve_cus=cfg.ag_reserve, ag=ag)
        # the ACK wait: the launch's first copy workgroup performs it (AG_WAIT_ACKS) and the op
        # stays in the plan for the simulator; otherwise a wait kernel / stream wait
        acks = [flags.ref("ACK", p) for p in range(d) if p != rank]
        if in_launch:
            for c in _chunks(acks):
                plan.wait_signal(S_MAIN, c, method=SIG_IN_LAUNCH)
        else:
            _wait(plan, S_MAIN, acks, cfg)
    elif alg == "coll_pipeline" and be == "ipc" and cfg.fused:
        # ONE flag-gated GEMM over all m rows instead of s stage GEMMs: tiles are dispatched
        # block-major (block 0 of the own shard and of every peer, then block 1, ...), the order
        # the chunked pulls land in, and each tile spins until its row block's ARRIVE flag is set
        # by the copy stream that pulled it; no stage boundaries, no per-stage GEMM tail.
        rows = ml // cfg.s
        peers = _peer_order(rank, d, cfg.ring)
        jobs = [(p, [(p * ml + j * rows, rows) for j in range(cfg.s)]) for p in peers]
        _ipc_pull_shards(plan, rank, d, cfg, flags, jobs, lambda r0: arow(r0), k * ein,
                         arrive_block=lambda p, b: flags.ref("ARRIVE", p * cfg.s + b))
        # enqueued after the pulls (every dependency points backwards in enqueue order)
        _signal(plan, S_MAIN, [flags.ref("ARRIVE", rank * cfg.s + j) for j in range(cfg.s)], cfg)
        gemm(S_MAIN, A, C, m, flags=flags.ref("ARRIVE", 0), flag_rows=rows, nshards=d * cfg.s,
             nsub=cfg.s, first_shard=rank, tile_order=1, reserve_cus=_gate_reserve(cfg))
        _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in range(d) if p != rank], cfg)
    elif alg == "coll_pipeline" and be == "ipc":
        rows = ml // cfg.s
        peers = _peer_order(rank, d, cfg.ring)
        jobs = [(p, [(p * ml + j * rows, rows) for j in range(cfg.s)]) for p in peers]

        def stage_gemm(j: int, done) -> None:  # right after chunk j of every peer is enqueued
            # (one event per block when one kernel / batch op moved every peer's chunk)
            for e in _unique(done[p][j] for p in peers):
                plan.wait(S_MAIN, e)
            gemm(S_MAIN, arow(j * rows), crow(j * rows), d * rows, a_grp=rows, a_gstride=ml,
                 c_grp=rows, c_gstride=ml)

        _ipc_pull_shards(plan, rank, d, cfg, flags, jobs, lambda r0: arow(r0), k * ein,
                         on_block=stage_gemm)
        _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in range(d) if p != rank], cfg)
    elif alg == "p2p_pipeline" and be == "ipc":
        order = _shard_order(rank, d, cfg.ring)
        peers = [p for p in order if p != rank]
        # the own shard's GEMM needs no transfer: enqueue it before the pulls (time order)
        own_first = (not cfg.fused) and order[0] == rank
        done = _ipc_pull_shards(plan, rank, d, cfg, flags, [(p, [(p * ml, ml)]) for p in peers],
                                lambda r0: arow(r0), k * ein,
                                arrive=flags.ref if cfg.fused else None,
                                after_ready=(lambda: shard_gemm(rank)) if own_first else None)
        if cfg.fused:
            _signal(plan, S_MAIN, [flags.ref("ARRIVE", rank)], cfg)
            gemm(S_MAIN, A, C, m, flags=flags.ref("ARRIVE", 0), flag_rows=ml, nshards=d,
                 first_shard=order[0], tile_order=1, reserve_cus=_gate_reserve(cfg))
        else:
            for p in order:
                if p == rank and own_first:
                    continue
                if p != rank:
                    plan.wait(S_MAIN, done[p][0])
                shard_gemm(p)
        _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in range(d) if p != rank], cfg)
    elif alg == "p2p_pipeline" and be == "rccl":
        # pairwise exchange steps: step j sends my shard to r-j, receives shard r+j
        evs = {}
        for j in range(1, d):
            to, frm = (rank - j) % d, (rank + j) % d
            plan.group_start(S_COMM)
            plan.send(S_COMM, arow(rank * ml), ml * k, comm_dt, to)
            plan.recv(S_COMM, arow(frm * ml), ml * k, comm_dt, frm)
            plan.group_end(S_COMM)
            e = plan.event()
            plan.record(S_COMM, e)
            evs[frm] = e
        for p in [(rank + j) % d for j in range(d)]:
            if p != rank:
                plan.wait(S_MAIN, evs[p])
            shard_gemm(p)
    else:  # pragma: no cover
        raise ValueError(f"unsupported combination {alg}/{be}")
    return plan, io


def _gemm_first(plan: Plan, cfg: AlgoConfig, producers=(S_COMM,)) -> bool:
    """Enqueue an RCCL-fed gated GEMM ahead of its producers? Only when its stream can never share
    an in-order hardware queue with theirs: HIP pools hardware queues per stream priority (the
    executor's stream-0 ops run on a normal-priority pool stream, the comm streams are created at
    high priority) and a CU-masked stream gets a queue of its own, so the GEMM's spinning tiles
    can then never sit in front of a collective or signal kernel that sets their flags.
    Otherwise (a producer on a normal-priority stream, or one hardware queue per process) the GEMM
    goes after the producers: correct in any queue mapping, at the cost of starting after the host
    has enqueued the collectives. The decision is recorded in ``plan.meta['gemm_first']``."""
    import os

    try:
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        queues = 4
    prio = plan.stream_priority
    separate = (cfg.comm_cus > 0 or
                all(p < len(prio) and prio[p] > 0 for p in producers) and prio[S_MAIN] == 0)
    first = bool(cfg.gemm_first and queues >= 2 and separate)
    plan.meta["gemm_first"] = first
    return first


def _rccl_gate(plan: Plan, cfg: AlgoConfig) -> int:
    """Reserve of an RCCL-fed gated GEMM and the CTA cap of the communicator feeding it: the
    collectives launch at most ``reserve`` workgroups (``rccl_max_ctas``, applied when the plan is
    bound: ``context.rccl_gate_cap``), so GEMM grid + RCCL grid <= num_cus by construction. With
    a CU split the collectives run on CUs of their own and keep RCCL's default."""
    reserve = _gate_reserve(cfg)
    plan.meta["rccl_max_ctas"] = 0 if cfg.comm_cus > 0 else reserve
    return reserve


def _col_rccl_fused_coll(plan, rank, d, m, n, k, ein, cfg, A, Bt, C, comm_dt, gdt) -> None:
    """coll_pipeline over RCCL feeding ONE persistent flag-gated GEMM over all m rows
    (``TPColumnwise/fuser.py:59-100`` semantics, SURVEY.md §7.3 hard part #1: at d = 8, s = 8 a
    stage GEMM is 8192 x n x k, 128 tiles of 256² for 256 CUs; the fused GEMM is the flagship's
    1024-tile persistent kernel).

    Stage j's ``ncclAllGather`` lands in a stage-major gather buffer G (block (j, p) = rank p's
    stage-j rows at G row (j*d + p)*rows); a signal kernel then raises ARRIVE[p*s + j] for every
    peer p (on the comm stream, or ``sig_side``: a third stream behind an event). The GEMM reads A
    through a row-block address table
    (logical block p*s + j = C rows p*m/d + j*rows: C keeps its canonical layout, no permutation)
    whose own blocks point at the rank's input shard itself, so the own tiles (dispatched first and
    never gated, tile_order 3: no signal op for them) run while stage 0 is still in flight. The
    flags are local (this rank's own signal kernels set them) and the gated GEMM leaves
    ``reserve_cus`` CUs to RCCL's kernels."""
    ml = m // d
    s = cfg.s
    rows = ml // s
    blk = rows * k * ein
    G = plan.buffer("G", m * k * ein)
    flags = _Flags(plan, d, s, symmetric=False)
    table = []
    for p in range(d):
        for j in range(s):
            table.append(A + (rank * ml + j * rows) * k * ein if p == rank
                         else G + (j * d + p) * blk)
    gemm = dict(M=m, N=n, K=k, lda=k, ldb=k, ldc=n, **gdt, a_shards=table, shard_rows=rows,
                flags=flags.ref("ARRIVE", 0), flag_rows=rows, nshards=d * s, nsub=s,
                first_shard=rank, tile_order=3, reserve_cus=_rccl_gate(plan, cfg))
    # the signal kernels run on the comm stream or, sig_side, on their own stream
    s_sig = 2 if cfg.sig_side else S_COMM
    first = _gemm_first(plan, cfg, (S_COMM, s_sig))
    if first:
        plan.gemm(S_MAIN, A, Bt, C, **gemm)
    for j in range(s):
        plan.allgather(S_COMM, A + (rank * ml + j * rows) * k * ein, G + j * d * blk, rows * k,
                       comm_dt)
        if cfg.sig_side:
            e = plan.event()
            plan.record(S_COMM, e)
            plan.wait(s_sig, e)
        # a kernel (release at system scope after the collective's kernel): the gated tiles
        # acquire the rows RCCL wrote; a stream memop has no such fence
        for c in _chunks([flags.ref("ARRIVE", p * s + j) for p in range(d) if p != rank]):
            plan.signal(s_sig, c, method=SIG_KERNEL)
    if not first:
        plan.gemm(S_MAIN, A, Bt, C, **gemm)


def _col_rccl_fused_p2p(plan, rank, d, m, n, k, ein, cfg, A, Bt, C, comm_dt, gdt) -> None:
    """p2p_pipeline over RCCL send / recv (``TPColumnwise/fuser.py:102-146``) feeding ONE
    flag-gated GEMM over all m rows: step j receives shard (r+j)%d into its rows of A and a
    signal kernel raises ARRIVE[(r+j)%d]; the tiles run shard by shard from the own one
    (tile_order 3: the own shard first and never gated, then (r+1)%d, ...: the order the steps
    deliver them); the GEMM is enqueued first when that is safe (:func:`_gemm_first`).

    A is read through a row-block table (shard p = rows p*m/d of A itself): tile_order 3's "own
    shard never gated" lives in the table-A (APAN) instantiation of the persistent kernel, and
    ARRIVE[rank] is never raised (with plain A rows the own tiles spun until the
    timeout). The launcher refuses tile_order 3 on any kernel that would gate the own shard."""
    ml = m // d
    flags = _Flags(plan, d, 1, symmetric=False)
    gemm = dict(M=m, N=n, K=k, lda=k, ldb=k, ldc=n, **gdt, flags=flags.ref("ARRIVE", 0),
                flag_rows=ml, nshards=d, first_shard=rank, tile_order=3,
                a_shards=[A + p * ml * k * ein for p in range(d)], shard_rows=ml,
                reserve_cus=_rccl_gate(plan, cfg))
    s_sig = 2 if cfg.sig_side else S_COMM  # (see _col_rccl_fused_coll)
    first = _gemm_first(plan, cfg, (S_COMM, s_sig))
    if first:
        plan.gemm(S_MAIN, A, Bt, C, **gemm)
    for j in range(1, d):
        to, frm = (rank - j) % d, (rank + j) % d
        plan.group_start(S_COMM)
        plan.send(S_COMM, A + rank * ml * k * ein, ml * k, comm_dt, to)
        plan.recv(S_COMM, A + frm * ml * k * ein, ml * k, comm_dt, frm)
        plan.group_end(S_COMM)
        if cfg.sig_side:
            e = plan.event()
            plan.record(S_COMM, e)
            plan.wait(s_sig, e)
        plan.signal(s_sig, [flags.ref("ARRIVE", frm)], method=SIG_KERNEL)
    if not first:
        plan.gemm(S_MAIN, A, Bt, C, **gemm)


def _col_push(plan, rank, d, ml, cfg, flags, arow, crow, gemm, row_bytes) -> None:
    """Push variant of the IPC all-gather: every rank WRITES its own shard into each peer's
    gather buffer (one copy queue per peer, so all d-1 links carry posted writes at once; a
    write over xGMI needs no round trip, a pull's read does), then raises the peer's arrival flag.

    Flags (peer-owned slots are written remotely, local ones are waited on):
      * READY[p] (default / p2p) or CHUNK[j*d + p] (coll stage j): p's rows are in my buffer;
      * ACK[p]: p finished the GEMMs that read the rows I pushed there in the previous epoch,
        so I may overwrite them (waited with delta -1 before every push: first epoch passes).
    The receiver's GEMM of shard / stage waits the arrival flags on the compute stream and the
    ACKs go out after the last GEMM, so no rank overwrites rows a peer is still reading."""
    alg = cfg.algorithm
    peers = _peer_order(rank, d, cfg.ring)
    s = cfg.s if alg == "coll_pipeline" else 1
    rows = ml // s
    own = rank * ml

    def arrived(p: int, j: int, owner: Optional[int] = None) -> Ref:
        return (flags.ref("CHUNK", j * d + p, owner) if alg == "coll_pipeline"
                else flags.ref("READY", p, owner))

    if cfg.protocol == "kernel":
        st = _s_copy(0)
        _wait(plan, st, [flags.ref("ACK", p) for p in peers], cfg, delta=-1)
        for j in range(s):
            segs = [(arow(own + j * rows).at(p), arow(own + j * rows), rows * row_bytes)
                    for p in peers]
            for i in range(0, len(segs), 8):
                plan.copy_multi(st, segs[i:i + 8], max_blocks=cfg.copy_blocks)
            _signal(plan, st, [arrived(rank, j, owner=p) for p in peers], cfg)
    else:
        prev_last = None
        for idx, p in enumerate(peers):
            st = _s_copy(0) if cfg.protocol == "batch_memcpy" else _s_copy(idx)
            if cfg.inter_stream_sync and prev_last is not None and cfg.protocol != "batch_memcpy":
                plan.wait(st, prev_last)
            _wait(plan, st, [flags.ref("ACK", p)], cfg, delta=-1)
            for j in range(s):
                plan.copy(st, arow(own + j * rows).at(p), arow(own + j * rows), rows * row_bytes,
                          method=COPY_ENGINE)
                _signal(plan, st, [arrived(rank, j, owner=p)], cfg)
            prev_last = plan.event()
            plan.record(st, prev_last)
    # receiver side, compute stream
    if alg == "default":
        _wait(plan, S_MAIN, [arrived(p, 0) for p in peers], cfg)
        gemm(S_MAIN, arow(0), crow(0), d * ml)
    elif alg == "coll_pipeline":
        for j in range(s):
            _wait(plan, S_MAIN, [arrived(p, j) for p in peers], cfg)
            gemm(S_MAIN, arow(j * rows), crow(j * rows), d * rows, a_grp=rows, a_gstride=ml,
                 c_grp=rows, c_gstride=ml)
    else:  # p2p_pipeline: own shard first, then shards in ring order as they arrive
        for p in _shard_order(rank, d, cfg.ring):
            if p != rank:
                _wait(plan, S_MAIN, [arrived(p, 0)], cfg)
            gemm(S_MAIN, arow(p * ml), crow(p * ml), ml)
    _signal(plan, S_MAIN, [flags.ref("ACK", rank, owner=p) for p in peers], cfg)


def _col_direct(plan, rank, d, m, n, k, din, dout, ein, eout, cfg, gdt) -> Plan:
    """Direct-access AG+GEMM: no all-gather at all. Every rank keeps only its own shard in a
    symmetric buffer; ONE GEMM launch reads row block p straight from rank p's HBM over xGMI
    (IPC-mapped pointers in a per-shard address table, LDS-DMA from peer memory), so the
    transfer is spread over all d-1 links at once and fully overlapped with the MFMA work, and
    no [m, k] gather buffer is written or read locally. READY: my shard is in place for this
    epoch; ACK: I finished reading yours (the owner may overwrite it afterwards)."""
    ml = m // d
    A_own = plan.buffer("A_own", ml * k * ein, symmetric=True)
    C = plan.buffer("C", m * n * eout)
    Bt = Ref("Bt")
    if d == 1:
        plan.gemm(S_MAIN, A_own, Bt, C, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, **gdt)
        return plan
    flags = _Flags(plan, d, 1)
    peers = [p for p in range(d) if p != rank]
    _signal(plan, S_MAIN, [flags.ref("READY", rank, owner=p) for p in peers], cfg)
    _wait(plan, S_MAIN, [flags.ref("READY", p) for p in peers], cfg)
    shards = [A_own.at(None if p == rank else p) for p in range(d)]
    plan.gemm(S_MAIN, A_own, Bt, C, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, a_shards=shards,
              shard_rows=ml, **gdt)
    _signal(plan, S_MAIN, [flags.ref("ACK", rank, owner=p) for p in peers], cfg)
    _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in peers], cfg)
    return plan


def _ipc_pull_shards(plan: Plan, rank: int, d: int, cfg: AlgoConfig, flags: _Flags,
                     jobs, row_ref, row_bytes: int, arrive=None, on_block=None, after_ready=None,
                     arrive_block=None):
    """Pull row blocks of the symmetric buffer from peers into the same rows locally.

    ``jobs`` = [(peer, [(row0, nrows), ...]), ...] in issue order, the same number of blocks per
    peer. Returns ``{peer: [event after block i]}``. Protocol: READY[peer] is waited before the
    first read of that peer; ACK is sent to the peer after the last block has landed (the peer
    may then overwrite its shard). Blocks are enqueued block-major (block i of every peer, then
    ``on_block(i, done)`` — e.g. the GEMM of stage i — then block i+1; see the module docstring
    on hardware-queue sharing); ``inter_stream_sync`` keeps the peer-major order it needs.
    ``after_ready()`` is enqueued right after this rank's READY signal, before any pull (e.g.
    the GEMM of the rank's own shard, which needs no transfer). ``arrive(name, p)`` is signalled
    after the last block of peer p, ``arrive_block(p, b)`` (a local flag) after each block.
    """
    _signal(plan, S_MAIN, [flags.ref("READY", rank, owner=p) for p in range(d) if p != rank], cfg)
    if after_ready is not None:
        after_ready()
    done: Dict[int, List[int]] = {}
    nblk = len(jobs[0][1])
    if cfg.protocol in ("kernel", "batch_memcpy") and not (
            cfg.protocol == "batch_memcpy" and cfg.inter_stream_sync):
        # ONE op per block index reading every peer: a CU copy kernel (copy_multi) or one
        # batched copy-engine submission (copy_batch = hipMemcpyBatchAsync), <= 8 segments each
        st = _s_copy(0)
        _wait(plan, st, [flags.ref("READY", p) for p, _ in jobs], cfg)
        for b in range(nblk):
            segs = []
            for p, blocks in jobs:
                r0, nr = blocks[b]
                segs.append((row_ref(r0), row_ref(r0).at(p), nr * row_bytes))
            for i in range(0, len(segs), 8):
                if cfg.protocol == "kernel":
                    plan.copy_multi(st, segs[i:i + 8], max_blocks=cfg.copy_blocks)
                else:
                    plan.copy_batch(st, segs[i:i + 8])
            if arrive_block is not None:
                _signal(plan, st, [arrive_block(p, b) for p, _ in jobs], cfg)
            e = plan.event()
            plan.record(st, e)
            for p, _ in jobs:
                done.setdefault(p, []).append(e)
            if on_block is not None:
                on_block(b, done)
        if arrive is not None:
            _signal(plan, st, [arrive("ARRIVE", p) for p, _ in jobs], cfg)
        _signal(plan, st, [flags.ref("ACK", rank, owner=p) for p, _ in jobs], cfg)
        return done

    split = max(cfg.copy_streams, 1) if cfg.protocol == "memcpy" else 1

    def stream_of(idx: int, part: int = 0) -> int:
        return _s_copy(0) if cfg.protocol == "batch_memcpy" else _s_copy(idx * split + part)

    def pull(idx: int, p: int, b: int) -> None:
        """Block b of peer p; with copy_streams > 1 its rows are split over that many streams
        (one copy engine each) and joined on the peer's first stream."""
        r0, nr = jobs[idx][1][b]
        st = stream_of(idx)
        if split > 1:
            cuts = [r0 + (nr * j) // split for j in range(split + 1)]
            for j in range(split):  # every part's copy first, then the join on part 0
                a0, a1 = cuts[j], cuts[j + 1]
                if a1 > a0:
                    plan.copy(stream_of(idx, j), row_ref(a0), row_ref(a0).at(p),
                              (a1 - a0) * row_bytes, method=COPY_ENGINE)
            for j in range(1, split):
                plan.edge(stream_of(idx, j), st)
        else:
            plan.copy(st, row_ref(r0), row_ref(r0).at(p), nr * row_bytes, method=COPY_ENGINE)
        if arrive_block is not None:
            _signal(plan, st, [arrive_block(p, b)], cfg)
        e = plan.event()
        plan.record(st, e)
        done.setdefault(p, []).append(e)

    def finish(idx: int, p: int) -> None:
        st = stream_of(idx)
        if arrive is not None:
            _signal(plan, st, [arrive("ARRIVE", p)], cfg)
        _signal(plan, st, [flags.ref("ACK", rank, owner=p)], cfg)

    if cfg.inter_stream_sync and cfg.protocol != "batch_memcpy":
        prev_last = None  # peer idx starts after peer idx-1's last block: peer-major issue
        for idx, (p, _) in enumerate(jobs):
            if prev_last is not None:
                plan.wait(stream_of(idx), prev_last)
            _wait(plan, stream_of(idx), [flags.ref("READY", p)], cfg)
            for b in range(nblk):
                pull(idx, p, b)
            prev_last = done[p][-1]
            finish(idx, p)
        if on_block is not None:
            for b in range(nblk):
                on_block(b, done)
        return done
    for idx, (p, _) in enumerate(jobs):
        for part in range(split):
            _wait(plan, stream_of(idx, part), [flags.ref("READY", p)], cfg)
    for b in range(nblk):
        for idx, (p, _) in enumerate(jobs):
            pull(idx, p, b)
        if on_block is not None:
            on_block(b, done)
    for idx, (p, _) in enumerate(jobs):
        finish(idx, p)
    return done


def _col_ag_after(plan, rank, d, m, n, k, ein, eout, dout, cfg, A, Bt, C, flags, gdt):
    ml = m // d
    comm_dt = dout

    def gemm(stream, r0, M):
        plan.gemm(stream, A + r0 * k * ein, Bt, C + r0 * n * eout, M=M, N=n, K=k, lda=k, ldb=k,
                  ldc=n, **gdt)

    if d == 1:
        gemm(S_MAIN, 0, m)
        return
    alg, be = cfg.algorithm, cfg.backend
    nch = cfg.s if alg == "coll_pipeline" else 1
    if alg == "coll_pipeline" and ml % nch:
        raise ValueError("m/d must be divisible by s")
    rows = ml // nch
    if be == "rccl":
        if alg == "default":
            gemm(S_MAIN, rank * ml, ml)
            plan.allgather(S_MAIN, C + rank * ml * n * eout, C, ml * n, comm_dt)
            return
        for j in range(nch):
            gemm(S_MAIN, rank * ml + j * rows, rows)
            plan.edge(S_MAIN, S_COMM)
            plan.group_start(S_COMM)
            for p in range(d):
                if p == rank:
                    continue
                plan.send(S_COMM, C + (rank * ml + j * rows) * n * eout, rows * n, comm_dt, p)
                plan.recv(S_COMM, C + (p * ml + j * rows) * n * eout, rows * n, comm_dt, p)
            plan.group_end(S_COMM)
        return
    # ipc: chunk-ready flags per chunk, peers pull the chunk rows of C
    peers = _peer_order(rank, d, cfg.ring)
    _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in peers], cfg, delta=-1)
    for j in range(nch):
        gemm(S_MAIN, rank * ml + j * rows, rows)
        _signal(plan, S_MAIN, [flags.ref("CHUNK", j * d + rank, owner=p) for p in peers], cfg)
    evs = []
    for idx, p in enumerate(peers):
        st = _s_copy(0) if cfg.protocol == "batch_memcpy" else _s_copy(idx)
        for j in range(nch):
            _wait(plan, st, [flags.ref("CHUNK", j * d + p)], cfg)
            r0 = p * ml + j * rows
            off = r0 * n * eout
            if cfg.protocol == "kernel":
                plan.copy(st, C + off, (C + off).at(p), rows * n * eout, method=COPY_KERNEL,
                          max_blocks=cfg.copy_blocks)
            else:
                plan.copy(st, C + off, (C + off).at(p), rows * n * eout)
        _signal(plan, st, [flags.ref("ACK", rank, owner=p)], cfg)
        e = plan.event()
        plan.record(st, e)
        evs.append(e)
    for e in evs:
        plan.wait(S_MAIN, e)


# =====================================================================================
#  TP-Rowwise
# =====================================================================================
def check_rowwise(d: int, m: int, n: int, k: int, cfg: AlgoConfig) -> None:
    if m % d or k % d:
        raise ValueError(f"m ({m}) and k ({k}) must be divisible by world_size ({d})")
    if cfg.algorithm == "coll_pipeline" and m % (d * cfg.s):
        raise ValueError(f"m ({m}) must be divisible by s*world_size ({cfg.s}*{d})")
    if cfg.algorithm not in ("default", "coll_pipeline", "p2p_pipeline"):
        raise ValueError(f"unknown algorithm {cfg.algorithm} for tp_rowwise")
    if cfg.backend not in ("rccl", "ipc"):
        raise ValueError(f"unknown backend {cfg.backend}")
    if cfg.direction != "pull":
        raise ValueError("direction=push is a tp_columnwise all-gather option (the rowwise "
                         "p2p_pipeline already pushes its partials)")
    if cfg.fused and not (cfg.algorithm == "p2p_pipeline" and cfg.backend == "ipc"):
        raise ValueError("fused=True for tp_rowwise is the direct-store p2p_pipeline (backend=ipc: "
                         "the GEMM epilogue writes each peer's partial into its receive slot); the "
                         "flag-gated GEMM over arriving rows is a tp_columnwise all-gather option")
    if d > 16:
        raise ValueError("at most 16 ranks per node are supported by the reduce op")


def build_tp_rowwise(rank: int, d: int, m: int, n: int, k: int, din: int, dout: int,
                     cfg: AlgoConfig) -> Tuple[Plan, PlanIO]:
    plan, io = _build_tp_rowwise(rank, d, m, n, k, din, dout, cfg)
    _finish(plan, cfg)
    return plan, io


def _build_tp_rowwise(rank: int, d: int, m: int, n: int, k: int, din: int, dout: int,
                      cfg: AlgoConfig) -> Tuple[Plan, PlanIO]:
    check_rowwise(d, m, n, k, cfg)
    ein, eout = DT_SIZE[din], DT_SIZE[dout]
    kl, ml = k // d, m // d
    plan = Plan(rank, d, nstreams=_nstreams(d), stream_priority=[0, 1] + [1] * max(d - 1, 1))
    plan.meta.update(primitive="tp_rowwise", algorithm=cfg.algorithm, backend=cfg.backend)
    A = plan.buffer("A", m * kl * ein)
    Bt = plan.buffer("Bt", n * kl * ein)
    OUT = plan.buffer("OUT", ml * n * eout)
    io = PlanIO(TensorLoc("A", 0, m, kl, din), TensorLoc("Bt", 0, n, kl, din),
                TensorLoc("OUT", 0, ml, n, dout))
    flags = _Flags(plan, d, max(cfg.s, 1)) if cfg.backend == "ipc" and d > 1 else None
    gdt = dict(din=din, dout=dout, tile=cfg.tile, mode=cfg.mode)
    blk = ml * n * eout   # bytes of one [m/d, n] output block

    def gemm(stream, a_row0, c_ref, M, **kw):
        plan.gemm(stream, A + a_row0 * kl * ein, Bt, c_ref, M=M, N=n, K=kl, lda=kl, ldb=kl, ldc=n,
                  **gdt, **kw)

    if d == 1:
        gemm(S_MAIN, 0, OUT, m)
        return plan, io
    alg, be = cfg.algorithm, cfg.backend
    peers = _peer_order(rank, d, cfg.ring)
    if alg == "default" and be == "rccl":
        P = plan.buffer("P", m * n * eout)
        gemm(S_MAIN, 0, P, m)
        plan.reduce_scatter(S_MAIN, P, OUT, ml * n, dout)
    elif alg == "default" and be == "ipc":
        P = plan.buffer("P", m * n * eout, symmetric=True)
        _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in peers], cfg, delta=-1)
        gemm(S_MAIN, 0, P, m)
        _signal(plan, S_MAIN, [flags.ref("READY", rank, owner=p) for p in peers], cfg)
        _wait(plan, S_MAIN, [flags.ref("READY", p) for p in peers], cfg)
        srcs = _row_gather_sources(plan, rank, d, cfg, P + rank * blk, blk, peers, "RCV")
        plan.reduce(S_MAIN, OUT, srcs, ml * n, dout)
        _signal(plan, S_MAIN, [flags.ref("ACK", rank, owner=p) for p in peers], cfg)
    elif alg == "coll_pipeline" and be == "rccl":
        rows = ml // cfg.s
        for j in range(cfg.s):
            stg = plan.buffer(f"STG{j}", d * rows * n * eout)
            gemm(S_MAIN, j * rows, stg, d * rows, a_grp=rows, a_gstride=ml)
            plan.edge(S_MAIN, S_COMM)
            plan.reduce_scatter(S_COMM, stg, OUT + j * rows * n * eout, rows * n, dout)
    elif alg == "coll_pipeline" and be == "ipc":
        rows = ml // cfg.s
        sblk = rows * n * eout
        for j in range(cfg.s):
            stg = plan.buffer(f"STG{j}", d * sblk, symmetric=True)
            _wait(plan, S_MAIN, [flags.ref("ACKS", j * d + p) for p in peers], cfg, delta=-1)
            gemm(S_MAIN, j * rows, stg, d * rows, a_grp=rows, a_gstride=ml)
            plan.edge(S_MAIN, S_COMM)
            _signal(plan, S_COMM, [flags.ref("CHUNK", j * d + rank, owner=p) for p in peers], cfg)
            _wait(plan, S_COMM, [flags.ref("CHUNK", j * d + p) for p in peers], cfg)
            srcs = [stg + rank * sblk] + [(stg + rank * sblk).at(p) for p in peers]
            plan.reduce(S_COMM, OUT + j * sblk, srcs, rows * n, dout)
            _signal(plan, S_COMM, [flags.ref("ACKS", j * d + rank, owner=p) for p in peers], cfg)
    elif alg == "p2p_pipeline" and be == "ipc" and cfg.fused:
        # Direct-store reduce-scatter: ONE GEMM over all m rows whose epilogue writes row block q
        # (the partial rank q reduces) straight into q's receive slot for this rank over xGMI
        # (csrc/gemm/gemm_kernels.h c_row); tile_order=2 interleaves the blocks, so the tiles in
        # flight store to every peer (every link) at once. No staging buffer, no copy engine,
        # no HBM round trip of the partials; the comm IS the GEMM's C stream.
        RECV = plan.buffer("RECV", d * blk, symmetric=True)
        _wait(plan, S_MAIN, [flags.ref("ACK", p) for p in peers], cfg, delta=-1)
        slots = [(RECV + rank * blk).at(q) if q != rank else RECV + rank * blk for q in range(d)]
        gemm(S_MAIN, 0, RECV + rank * blk, m, c_shards=slots, c_shard_rows=ml, nshards=d,
             tile_order=2)
        # READY always from the signal kernel: its system-scope release fence orders the GEMM's
        # remote C stores (over xGMI, into the peers' RECV) before the flag, whatever cfg.signal
        # says (a stream memop has no such fence for stores another kernel issued)
        for c in _chunks([flags.ref("READY", rank, owner=p) for p in peers]):
            plan.signal(S_MAIN, c, method=SIG_KERNEL)
        _wait(plan, S_MAIN, [flags.ref("READY", p) for p in peers], cfg)
        plan.reduce(S_MAIN, OUT, [RECV + q * blk for q in range(d)], ml * n, dout)
        _signal(plan, S_MAIN, [flags.ref("ACK", rank, owner=p) for p in peers], cfg)
    elif alg == "p2p_pipeline" and be == "ipc":
        PST = plan.buffer("PST", d * blk)
        RECV = plan.buffer("RECV", d * blk, symmetric=True)
        evs = {}
        for p in peers:                        # peers' partials first, shipped as they finish
            gemm(S_MAIN, p * ml, PST + p * blk, ml)
            e = plan.event()
            plan.record(S_MAIN, e)
            evs[p] = e
        prev = None
        for idx, p in enumerate(peers):
            st = _s_copy(0) if cfg.protocol == "batch_memcpy" else _s_copy(idx)
            plan.wait(st, evs[p])
            if cfg.inter_stream_sync and prev is not None and cfg.protocol != "batch_memcpy":
                plan.wait(st, prev)
            _wait(plan, st, [flags.ref("ACK", p)], cfg, delta=-1)
            method = COPY_KERNEL if cfg.protocol == "kernel" else COPY_ENGINE
            plan.copy(st, (RECV + rank * blk).at(p), PST + p * blk, blk, method=method,
                      max_blocks=cfg.copy_blocks)
            _signal(plan, st, [flags.ref("READY", rank, owner=p)], cfg)
            prev = plan.event()
            plan.record(st, prev)
        gemm(S_MAIN, rank * ml, RECV + rank * blk, ml)   # own block last, straight into RECV
        _wait(plan, S_MAIN, [flags.ref("READY", p) for p in peers], cfg)
        plan.reduce(S_MAIN, OUT, [RECV + q * blk for q in range(d)], ml * n, dout)
        _signal(plan, S_MAIN, [flags.ref("ACK", rank, owner=p) for p in peers], cfg)
    elif alg == "p2p_pipeline" and be == "rccl":
        PST = plan.buffer("PST", d * blk)
        RECV = plan.buffer("RECV", d * blk)
        evs = {}
        for j in range(1, d):
            dst = (rank + j) % d
            gemm(S_MAIN, dst * ml, PST + dst * blk, ml)
            e = plan.event()
            plan.record(S_MAIN, e)
            evs[j] = e
        for j in range(1, d):
            to, frm = (rank + j) % d, (rank - j) % d
            plan.wait(S_COMM, evs[j])
            plan.group_start(S_COMM)
            plan.send(S_COMM, PST + to * blk, ml * n, dout, to)
            plan.recv(S_COMM, RECV + frm * blk, ml * n, dout, frm)
            plan.group_end(S_COMM)
        gemm(S_MAIN, rank * ml, RECV + rank * blk, ml)
        plan.edge(S_COMM, S_MAIN)
        plan.reduce(S_MAIN, OUT, [RECV + q * blk for q in range(d)], ml * n, dout)
    else:  # pragma: no cover
        raise ValueError(f"unsupported combination {alg}/{be}")
    return plan, io


def _row_gather_sources(plan, rank, d, cfg, own_ref, blk, peers, stage_name):
    """Sources of this rank's output block: direct peer reads (kernel) or SDMA pulls (memcpy)."""
    if cfg.protocol == "kernel":
        return [own_ref] + [own_ref.at(p) for p in peers]
    R = plan.buffer(stage_name, d * blk)
    if cfg.protocol == "batch_memcpy":  # every peer's block in one batched submission
        st = _s_copy(0)
        plan.edge(S_MAIN, st)
        segs = [(R + p * blk, own_ref.at(p), blk) for p in peers]
        for i in range(0, len(segs), 8):
            plan.copy_batch(st, segs[i:i + 8])
        plan.edge(st, S_MAIN)
        return [own_ref] + [R + p * blk for p in peers]
    evs = []
    for idx, p in enumerate(peers):
        st = _s_copy(0) if cfg.protocol == "batch_memcpy" else _s_copy(idx)
        plan.edge(S_MAIN, st)
        plan.copy(st, R + p * blk, own_ref.at(p), blk)
        e = plan.event()
        plan.record(st, e)
        evs.append(e)
    for e in evs:
        plan.wait(S_MAIN, e)
    return [own_ref] + [R + p * blk for p in peers]
