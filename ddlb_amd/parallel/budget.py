"""Per-rank budget of an N>1 plan on ONE GPU: what rank 0 of a d-rank job computes, copies and
enqueues, replayed locally (VERDICT r3 "next round" #2).

The reference's timed region is one ``impl.run()`` per iteration (``ddlb/benchmark.py:127-186``);
at d = 8 that holds the stage GEMMs, the communication and the per-op host work of the plan. A
one-GPU box cannot run the job, but it can run everything rank 0 does to ITS device:

* the GEMMs with their exact shapes, grouped rows, row tables, tiles and flags (the flags are
  pre-set to a huge epoch, so every gate / wait passes as soon as it is reached);
* every transfer as a local copy of the same byte count on the same stream and by the same
  engine: pulls / pushes over xGMI read or write a local "shadow" of the peer's buffer (copy
  engines stay copy engines, CU copies stay CU copies), an RCCL all-gather becomes a CU copy of
  its d x count bytes (RCCL moves data with CU kernels), a reduce-scatter a d-way reduce kernel,
  a receive a CU copy of its bytes;
* every signal / wait / event op as enqueued (their host and GPU cost is part of the budget).

:func:`emulate` rewrites a rank's :class:`~ddlb_amd.parallel.plan.Plan` into that one-rank form;
:func:`gemm_only` keeps just its GEMMs, serialized on stream 0 and ungated. The result is an
EMULATED budget: HBM-local copies are faster than xGMI links and no peer is ever late, so it is a
lower bound on rank 0's time and never a scaling value.
"""

from __future__ import annotations

from typing import Dict, Optional

from ddlb_amd.parallel.plan import (COPY_KERNEL, DT_SIZE, OP_ALLGATHER, OP_COPY, OP_COPY_BATCH,
                                    OP_COPY_MULTI, OP_GEMM, OP_GROUP_END, OP_GROUP_START,
                                    OP_RECV, OP_REDUCE, OP_REDUCE_SCATTER, OP_SEND, OP_SIGNAL,
                                    OP_WAIT_SIGNAL, BufferSpec, Op, Plan, Ref)

SHADOW = "@peer"          # suffix of a symmetric buffer's local stand-in for the peers' copies
RCCL_SRC = "__rccl_src"   # source of the emulated RCCL transfers
PRESET = 0x7FFFFFF0       # flag words start here: every epoch wait passes on arrival


def _map(plan: Plan, ref: Optional[Ref]) -> Optional[Ref]:
    if ref is None:
        return None
    if ref.owner is None or ref.owner == plan.rank:
        return Ref(ref.buf, ref.off)
    return Ref(ref.buf + SHADOW, ref.off)


def _map_list(plan: Plan, refs):
    return None if refs is None else [_map(plan, r) for r in refs]


def emulate(plan: Plan, rccl_blocks: int = 32) -> Plan:
    """One-rank form of ``plan`` (see the module docstring). ``rccl_blocks``: CU budget of the
    copy kernels standing in for RCCL's kernels, never above the plan's own RCCL CTA cap (an
    RCCL-fed gated GEMM's communicator launches at most ``meta['rccl_max_ctas']`` workgroups)."""
    d = plan.world
    cap = int(plan.meta.get("rccl_max_ctas", 0))
    if cap > 0:
        rccl_blocks = min(rccl_blocks, cap)
    ep = Plan(0, 1, nstreams=plan.nstreams, stream_priority=list(plan.stream_priority))
    ep.meta = dict(plan.meta, emulated_world=d, emulated_rank=plan.rank)
    ep.nevents = plan.nevents
    for name, spec in plan.buffers.items():
        table = _map_list(plan, spec.table)
        ep.buffers[name] = BufferSpec(name, spec.nbytes, False, spec.zero, table)
        if spec.symmetric:
            ep.buffers[name + SHADOW] = BufferSpec(name + SHADOW, spec.nbytes, False, spec.zero)
    rccl_bytes = 16
    for op in plan.ops:
        a = op.args
        if op.kind in (OP_ALLGATHER, OP_REDUCE_SCATTER):
            rccl_bytes = max(rccl_bytes, d * a["count"] * DT_SIZE[a["dtype"]])
        elif op.kind in (OP_SEND, OP_RECV):
            rccl_bytes = max(rccl_bytes, a["count"] * DT_SIZE[a["dtype"]])
    if any(op.kind in (OP_ALLGATHER, OP_RECV) for op in plan.ops):
        ep.buffers[RCCL_SRC] = BufferSpec(RCCL_SRC, rccl_bytes)
    for op in plan.ops:
        a, k, st = op.args, op.kind, op.stream
        if k in (OP_GROUP_START, OP_GROUP_END, OP_SEND):
            continue
        if k == OP_ALLGATHER:
            nb = d * a["count"] * DT_SIZE[a["dtype"]]
            ep.copy(st, _map(plan, a["recv"]), Ref(RCCL_SRC), nb, method=COPY_KERNEL,
                    max_blocks=rccl_blocks)
            continue
        if k == OP_RECV:
            ep.copy(st, _map(plan, a["buf"]), Ref(RCCL_SRC), a["count"] * DT_SIZE[a["dtype"]],
                    method=COPY_KERNEL, max_blocks=rccl_blocks)
            continue
        if k == OP_REDUCE_SCATTER:
            es = DT_SIZE[a["dtype"]]
            send = _map(plan, a["send"])
            srcs = [send + i * a["count"] * es for i in range(d)]
            for i in range(0, len(srcs), 16):  # the reduce op takes <= 16 sources
                ep.reduce(st, _map(plan, a["recv"]), srcs[i:i + 16], a["count"], a["dtype"])
            continue
        na: Dict = {}
        for key, v in a.items():
            if isinstance(v, Ref):
                na[key] = _map(plan, v)
            elif isinstance(v, list) and v and isinstance(v[0], Ref):
                na[key] = _map_list(plan, v)
            elif key == "segs":
                na[key] = [(_map(plan, x), _map(plan, y), n) for x, y, n in v]
            elif key == "ag" and v is not None:
                g = dict(v)
                for gk in ("src", "ack", "wait_acks"):
                    if g.get(gk) is not None:
                        g[gk] = _map_list(plan, g[gk])
                for gk in ("ready", "count", "table"):
                    if g.get(gk) is not None:
                        g[gk] = _map(plan, g[gk])
                na[key] = g
            else:
                na[key] = v
        ep.ops.append(Op(k, st, na))
    return ep


def gemm_only(plan: Plan) -> Plan:
    """Just the GEMMs of an (emulated) plan, in issue order on stream 0, ungated (no flags, no
    in-kernel copies): the compute floor of the rank's schedule."""
    gp = Plan(0, 1, nstreams=1, stream_priority=[0])
    gp.meta = dict(plan.meta, gemm_only=True)
    for name, spec in plan.buffers.items():
        gp.buffers[name] = BufferSpec(name, spec.nbytes, False, spec.zero, spec.table)
    for op in plan.ops:
        if op.kind != OP_GEMM:
            continue
        a = dict(op.args, flags=None, ag=None)
        if a.get("tile_order") == 3:  # own-first order means "own rows ungated": plain order
            a["tile_order"] = 0
        gp.ops.append(Op(OP_GEMM, 0, a))
    return gp


def flag_buffers(plan: Plan):
    """Names of the zero-initialised buffers of an emulated plan that hold flag words (to be
    pre-set to :data:`PRESET` before the runs)."""
    return [n for n, s in plan.buffers.items() if s.zero]


def op_counts(plan: Plan) -> Dict[str, int]:
    from ddlb_amd.parallel.plan import OP_NAMES

    out: Dict[str, int] = {}
    for op in plan.ops:
        out[OP_NAMES[op.kind]] = out.get(OP_NAMES[op.kind], 0) + 1
    return out


def signal_ops(plan: Plan) -> int:
    return sum(1 for op in plan.ops if op.kind in (OP_SIGNAL, OP_WAIT_SIGNAL))


def copy_bytes(plan: Plan) -> int:
    total = 0
    for op in plan.ops:
        if op.kind == OP_COPY:
            total += op.args["nbytes"]
        elif op.kind in (OP_COPY_MULTI, OP_COPY_BATCH):
            total += sum(n for _, _, n in op.args["segs"])
        elif op.kind == OP_REDUCE:
            total += op.args["count"] * DT_SIZE[op.args["dtype"]] * len(op.args["srcs"])
    return total


def link_bytes(plan: Plan) -> Dict[int, int]:
    """Bytes each peer's link carries in ONE direction in one run of rank ``plan.rank``'s ORIGINAL
    (not emulated) plan (what it receives, or sends for pushes and direct stores): pulls / pushes
    by copy engines or CU copies, RCCL
    collectives and send / recv (full-mesh model: an all-gather or reduce-scatter of ``count``
    elements per rank moves ``count`` to and from every peer), the in-kernel all-gather's row
    blocks, a direct-access GEMM's peer shards (read once: the re-reads of an A panel by the
    tiles of other N columns are assumed to hit the local L2) and a direct-store GEMM's peer row
    blocks. A model for ranking candidates against a link budget, not a measurement."""
    from ddlb_amd.parallel.plan import OP_ALLGATHER, OP_REDUCE_SCATTER, OP_RECV, OP_SEND

    me = plan.rank
    out: Dict[int, int] = {p: 0 for p in range(plan.world) if p != me}

    def peer(ref: Optional[Ref]) -> Optional[int]:
        return ref.owner if ref is not None and ref.owner not in (None, me) else None

    for op in plan.ops:
        a, k = op.args, op.kind
        if k == OP_COPY:
            p = peer(a["src"]) if peer(a["src"]) is not None else peer(a["dst"])
            if p is not None:
                out[p] += a["nbytes"]
        elif k in (OP_COPY_MULTI, OP_COPY_BATCH):
            for dst, src, n in a["segs"]:
                p = peer(src) if peer(src) is not None else peer(dst)
                if p is not None:
                    out[p] += n
        elif k in (OP_ALLGATHER, OP_REDUCE_SCATTER):
            for p in out:
                out[p] += a["count"] * DT_SIZE[a["dtype"]]
        elif k in (OP_SEND, OP_RECV):
            if a["peer"] in out:
                out[a["peer"]] += a["count"] * DT_SIZE[a["dtype"]]
        elif k == OP_REDUCE:
            for src in a["srcs"]:
                p = peer(src)
                if p is not None:
                    out[p] += a["count"] * DT_SIZE[a["dtype"]]
        elif k == OP_GEMM:
            es, eo = DT_SIZE[a["din"]], DT_SIZE[a["dout"]]
            g = a.get("ag")
            if g is not None:
                npro, nsub = a["nshards"] // a["nsub"], a["nsub"]
                for q in range(npro):
                    if q != g["rank"] and q in out:
                        out[q] += nsub * a["flag_rows"] * a["lda"] * es
            for i, ref in enumerate(a.get("a_shards") or []):
                p = peer(ref)
                if p is not None:
                    rows = min(a["shard_rows"], a["M"] - i * a["shard_rows"])
                    out[p] += max(rows, 0) * a["K"] * es
            for i, ref in enumerate(a.get("c_shards") or []):
                p = peer(ref)
                if p is not None:
                    rows = min(a["c_shard_rows"], a["M"] - i * a["c_shard_rows"])
                    out[p] += max(rows, 0) * a["N"] * eo
    return out
