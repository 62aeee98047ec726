"""First-contact diagnostics of the N>1 data plane, for ``bench.py`` at world > 1.

The first multi-GPU run of this framework is the driver's own 8-GPU scaling bench. If its
number is poor, the JSON line must say why, within a bounded time. Three parts, each in the same
child process (one HIP context, one rendezvous), each guarded and timed:

``xgmi``   per-peer pull bandwidth over xGMI at the plan's shard size: the copy engine
           (``hipMemcpyAsync`` from the peer's IPC-mapped shard) and a CU copy kernel, one peer
           at a time in ring order (step j: every rank pulls from rank + j, so each link
           direction carries one transfer) and from all d - 1 peers at once, in GB/s
``rccl``   RCCL all-gather / reduce-scatter bus bandwidth at the plans' message sizes (the
           default all-gather's whole shard, a coll_pipeline stage's slice, the rowwise
           reduce-scatter block) on the default communicator and on the one capped at the fused
           plans' CTA cap: what the cap costs
``trace``  one per-op GPU timeline of the final winner (the executor's event stamps): the GEMM
           spans against the transfer / collective spans, and which stream ends last

The reference's own diagnostics stop at a per-iteration time MAX-reduced over ranks
(``/root/reference/ddlb/benchmark.py:190-204``); its users read NCCL's busbw tables
(``/root/reference/README.md:141-145``) from separate tools.
"""

from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

PARTS = ("xgmi", "rccl", "trace")


def message_sizes(primitive: str, m: int, n: int, k: int, d: int, esz: int) -> Dict[str, int]:
    """Per-rank message bytes of the plans at this shape (labels -> bytes)."""
    if primitive == "tp_rowwise":
        blk = m // d * n * 2  # bf16 partial block each rank receives (reduce-scatter output)
        return {"rs_block": blk, "rs_block_s4": blk // 4}
    shard = m // d * k * esz  # the all-gather's shard
    return {"ag_shard": shard, "ag_stage_s4": shard // 4, "ag_stage_s8": shard // 8}


def run(parts: Dict[str, Callable[[], Dict]], budget_s: float,
        clock: Callable[[], float] = time.perf_counter) -> Dict:
    """Run the parts in order within ``budget_s``: a part that raises is reported with its error,
    a part that would start past the budget is skipped; every part's wall time is recorded."""
    out: Dict = {"budget_s": budget_s}
    t0 = clock()
    for name, fn in parts.items():
        if clock() - t0 > budget_s:
            out[name] = {"skipped": f"budget {budget_s:.0f} s spent"}
            continue
        t1 = clock()
        try:
            res = fn()
        except Exception as e:  # reported, never raised: the other parts still run
            res = {"error": f"{type(e).__name__}: {str(e).splitlines()[0][:200]}"
                   if str(e) else type(e).__name__}
        res["wall_s"] = round(clock() - t1, 2)
        out[name] = res
    out["wall_s"] = round(clock() - t0, 2)
    return out


def _time_ms(stream, fn, reps: int) -> float:
    """Mean ms of ``fn`` enqueued ``reps`` times on ``stream`` (one warm call first)."""
    import torch

    fn()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(stream)
    for _ in range(reps):
        fn()
    end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / reps


def xgmi_probe(comm, nbytes: int, reps: int = 3) -> Dict:
    """Per-peer copy-engine and CU-copy pull bandwidth (GB/s) of ``nbytes`` from each peer's
    IPC-mapped shard; one peer at a time (ring order) and every peer at once."""
    import torch

    r, d, dev = comm.rank, comm.world_size, comm.device
    if d < 2:
        return {"peers": 0}
    ctx = comm.native()
    C = ctx.C
    X = ctx.symmetric(nbytes)
    X.tensor.view(torch.uint8).fill_(r + 1)
    recv = torch.empty((d, nbytes), dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(d)]
    main = torch.cuda.current_stream(dev)
    gbs = lambda ms: round(nbytes / (ms * 1e-3) / 1e9, 1)  # noqa: E731
    one_sdma: Dict[str, float] = {}
    one_cu: Dict[str, float] = {}
    try:
        torch.cuda.synchronize(dev)
        comm.barrier()
        for j in range(1, d):
            p = (r + j) % d
            src, dst = X.ptr(p), recv[p].data_ptr()
            comm.barrier()
            ms = _time_ms(main, lambda: C.memcpy_async(dst, src, nbytes, main.cuda_stream), reps)
            one_sdma[str(p)] = gbs(ms)
            comm.barrier()
            ms = _time_ms(main, lambda: C.copy(dst, src, nbytes, 256, main.cuda_stream), reps)
            one_cu[str(p)] = gbs(ms)
        peers = [p for p in range(d) if p != r]
        ok = all(int(recv[p][0]) == p + 1 and int(recv[p][-1]) == p + 1 for p in peers)

        def all_sdma():
            ev = torch.cuda.Event()
            ev.record(main)
            for i, p in enumerate(peers):
                streams[i].wait_event(ev)
                C.memcpy_async(recv[p].data_ptr(), X.ptr(p), nbytes, streams[i].cuda_stream)
            for i in range(len(peers)):
                e = torch.cuda.Event()
                e.record(streams[i])
                main.wait_event(e)

        comm.barrier()
        ms_all_sdma = _time_ms(main, all_sdma, reps)
        segs = [(recv[p].data_ptr(), X.ptr(p), nbytes) for p in peers]

        def all_cu():
            for i in range(0, len(segs), 8):
                C.copy_multi(segs[i:i + 8], 256, main.cuda_stream)

        comm.barrier()
        ms_all_cu = _time_ms(main, all_cu, reps)
        torch.cuda.synchronize(dev)
        comm.barrier()
        tot = nbytes * len(peers)
        return {"bytes": nbytes, "sdma_one_GBps": one_sdma, "cu_one_GBps": one_cu,
                "sdma_all_GBps": round(tot / (ms_all_sdma * 1e-3) / 1e9, 1),
                "cu_all_GBps": round(tot / (ms_all_cu * 1e-3) / 1e9, 1), "bytes_ok": ok}
    finally:
        torch.cuda.synchronize(dev)
        ctx.release_symmetric([X])


def rccl_busbw(comm, sizes: Dict[str, int], caps=(0,), reps: int = 5) -> Dict:
    """Bus bandwidth (GB/s, NCCL's convention: algbw (d - 1) / d) of our communicator's
    all-gather (the ``ag_*`` sizes: bytes per rank) and reduce-scatter (``rs_*``: bf16 bytes
    each rank receives), per CTA cap (0 = RCCL's default)."""
    import torch

    from ddlb_amd.parallel.plan import DT_BF16, DT_U8

    d, dev = comm.world_size, comm.device
    ctx = comm.native()
    st = torch.cuda.Stream(dev, priority=-1)
    out: Dict[str, Dict[str, float]] = {}
    biggest = max(sizes.values())
    send = torch.zeros(d * biggest, dtype=torch.uint8, device=dev)
    recv = torch.zeros(d * biggest, dtype=torch.uint8, device=dev)
    for cap in caps:
        rc = ctx.rccl(cap)
        res: Dict[str, float] = {}
        for label, nb in sizes.items():
            if label.startswith("rs"):
                count = nb // 2
                fn = lambda: rc.reduce_scatter(send.data_ptr(), recv.data_ptr(), count,  # noqa
                                               DT_BF16, st.cuda_stream)
            else:
                fn = lambda: rc.all_gather(send.data_ptr(), recv.data_ptr(), nb, DT_U8,  # noqa
                                           st.cuda_stream)
            torch.cuda.synchronize(dev)
            comm.barrier()
            ms = _time_ms(st, fn, reps)
            alg = d * nb / (ms * 1e-3) / 1e9
            res[label] = round(alg * (d - 1) / d, 1) if d > 1 else round(alg, 1)
        out["default" if cap == 0 else f"cap{cap}"] = res
    torch.cuda.synchronize(dev)
    comm.barrier()
    return {"busbw_GBps": out, "sizes": sizes}


def winner_trace(impl, max_ops: int = 48) -> Dict:
    """Per-op GPU timeline of one run of a built native implementation (eager: per-op events
    need the executor's enqueue, not a replayed graph): GEMM time against transfer time, the
    span, and the ops that end last."""
    import torch

    bound = getattr(impl, "bound", None)
    if bound is None:
        return {"skipped": "not a native plan"}
    if bound.ex.graph_enabled():
        return {"skipped": "graph replay (no per-op events inside a replayed graph)"}
    bound.set_timeline(True)
    try:
        impl.run()
        torch.cuda.synchronize()
        rows = bound.timeline()
    finally:
        bound.set_timeline(False)
    span = max((r["end_ms"] for r in rows), default=0.0)
    kinds: Dict[str, float] = {}
    for r in rows:
        kind = r["op"].split()[0]
        kinds[kind] = kinds.get(kind, 0.0) + (r["end_ms"] - r["start_ms"])
    last = sorted(rows, key=lambda r: -r["end_ms"])[:3]
    ops: List[List] = [[r["op"], r["stream"], round(r["start_ms"], 4), round(r["end_ms"], 4)]
                       for r in rows[:max_ops]]
    return {"span_ms": round(span, 4), "busy_ms_by_kind": {k: round(v, 4) for k, v in
                                                          kinds.items()},
            "last_ops": [[r["op"], r["stream"], round(r["end_ms"], 4)] for r in last],
            "ops": ops, "nops": len(rows)}


def diagnose(comm, primitive: str, m: int, n: int, k: int, esz: int, impl_factory,
             budget_s: float = 30.0, caps=(0, 32), parts=PARTS) -> Dict:
    """All parts on this rank within ``budget_s`` (see the module docstring)."""
    d = comm.world_size
    sizes = message_sizes(primitive, m, n, k, d, esz)
    shard = m // d * (n if primitive == "tp_rowwise" else k) * (2 if primitive == "tp_rowwise"
                                                                 else esz)
    todo: Dict[str, Callable[[], Dict]] = {}
    if "xgmi" in parts:
        todo["xgmi"] = lambda: xgmi_probe(comm, shard)
    if "rccl" in parts:
        todo["rccl"] = lambda: rccl_busbw(comm, sizes, caps=caps)

    def trace() -> Dict:
        impl = impl_factory()
        try:
            for _ in range(3):
                impl.run()
            return winner_trace(impl)
        finally:
            impl.close()

    if "trace" in parts:
        todo["trace"] = trace
    return run(todo, budget_s)


def merge_ranks(per_rank: List[Optional[Dict]]) -> Dict:
    """One JSON record for the job: rank 0's RCCL and trace parts, every rank's xGMI probe."""
    base = dict(per_rank[0] or {})
    xg = [r.get("xgmi") if r else None for r in per_rank]
    if any(x for x in xg):
        base["xgmi"] = {str(i): x for i, x in enumerate(xg)}
    return base
