"""Multi-GPU preflight: is the N>1 data plane of THIS node sound, before a benchmark spends time on it?

The reference's product is ``mpirun -np N`` runs on real GPUs (``/root/reference/README.md:80-88``),
each child building its NCCL process group (``ddlb/primitives/TPColumnwise/pytorch.py:53-59``).
Here every N>1 path runs on mechanisms a shared-GPU rehearsal cannot exercise (RCCL at world > 1,
IPC peer memory and flag words over xGMI), so ``bench.py`` runs these checks once per job, each in
its own time-limited child, and drops the candidate families that fail:

==============  ==================================================================================
check           what it proves (every rank, every peer, two epochs)
==============  ==================================================================================
``torch_nccl``  torch's RCCL process group (the ``pytorch`` slot and the control plane): a SUM
                all-reduce of rank-dependent integers
``rccl``        our own ``ncclComm_t`` (``NativeContext.rccl``) on our streams: an all-gather of a
                byte pattern and an f32 reduce-scatter, compared bytewise
``ipc``         IPC mapping of symmetric buffers + the READY/ACK epoch handshake with every peer,
                with stream-memop signals (``hipStreamWriteValue32`` / ``WaitValue32``)
``ipc_ksig``    the same handshake with the signal / wait kernels (system-scope release, the
                form graph replay and ``signal=kernel`` use)
``ipc_kernel``  CU-copy pull (``copy_multi``: peer HBM read by a kernel over xGMI) of every
                peer's pattern, then a flag, then a read-back check
``ipc_sdma``    copy-engine pull (``hipMemcpyAsync`` from IPC-mapped peer memory, one stream per
                peer) of every peer's pattern
``ipc_push``    copy-engine push (posted writes into each peer's receive slot) + DONE flag
``ipc_batch``   every peer's pattern pulled in ONE batched submission (``hipMemcpyBatchAsync``,
                or where this HIP runtime lacks it, one launch of a graph of independent
                memcpy nodes); fails if the copies went out one by one
``ipc_agk``     the in-kernel all-gather: ONE gated persistent GEMM launch whose copy workgroups
                pull every peer's row blocks over xGMI (write-through publication, agent-scope
                gate acquire, ACK stores across the link), validated against fp32
``ipc_dstore``  the direct-store epilogue: a GEMM whose C row blocks are written straight into
                every peer's receive slot (tp_rowwise p2p fused), then the d-way reduce, validated
``rccl_cap``    the CTA cap the RCCL-fed gated GEMM relies on, OBSERVED: every CU but ``cap`` is
                held the way the gated GEMM holds it (one 512-thread workgroup per CU, the full
                register file and LDS, spinning), then an all-gather on the communicator capped
                at ``cap`` workgroups must finish on the CUs left free within a bound; it is
                timed against the same all-gather with nothing held. A collective that needs
                more CUs than the cap, or cannot run where the held CUs leave room, fails this
                phase (the holders are released by the host, so it never hangs) and drops the
                RCCL-fed fused family -- the communicator's own ``max_ctas`` is only what we
                asked RCCL for
``rccl_fused``  RCCL stage all-gathers feeding ONE flag-gated GEMM through signal kernels on the
                comm stream (coll_pipeline backend=rccl fused=True), validated
==============  ==================================================================================

The last three run the real plan builders through the primitives at a small shape (every tile
of the persistent 256x256 kernel, 2 epochs), so a mechanism that corrupts data over the link, not
only one that hangs, drops its candidate family.

Every check is a :class:`~ddlb_amd.parallel.plan.Plan` executed by the native executor, so the
same plans run on the CPU simulator in the tests (``tests/test_preflight.py``). A check that hangs
(a flag that never arrives over the link) leaves its phase missing from the progress file the
child rewrites after each phase; the parent reports it as ``failed: timeout``.
"""

from __future__ import annotations

import json
import os
import time
from typing import Callable, Dict, List, Optional

from ddlb_amd.parallel.plan import (COPY_ENGINE, DT_F32, DT_U8, SIG_KERNEL, SIG_STREAM, Plan,
                                    Ref)

IPC_PHASES = ("ipc", "ipc_ksig", "ipc_kernel", "ipc_sdma", "ipc_push", "ipc_batch", "ipc_agk",
              "ipc_dstore")
RCCL_PHASES = ("torch_nccl", "rccl", "rccl_cap", "rccl_fused", "rccl_fused_cm")
# phases that run a whole primitive (the real plan builder) instead of a data-movement plan:
# (primitive, options); the shape is PRIMITIVE_SHAPE(d)
PRIMITIVE_PHASES = {
    "ipc_agk": ("tp_columnwise", dict(algorithm="coll_pipeline", backend="ipc",
                                      multicast_protocol="kernel", fused=True, s=2,
                                      copy_blocks=16)),
    "ipc_dstore": ("tp_rowwise", dict(algorithm="p2p_pipeline", backend="ipc", fused=True,
                                      tile="pt4")),
    # tile pt4 (ipc_dstore, rccl_fused): the kernel the bench's candidates run at their shapes
    # (auto would pick the non-persistent t8 for these few tiles)
    "rccl_fused": ("tp_columnwise", dict(algorithm="coll_pipeline", backend="rccl", fused=True,
                                         s=2, tile="pt4")),
    # the same with a CU split: RCCL and the signal kernels on 32 CUs of their own, the gated GEMM
    # on the complement (a collective with more workgroups than the reserve cannot starve then)
    "rccl_fused_cm": ("tp_columnwise", dict(algorithm="coll_pipeline", backend="rccl", fused=True,
                                            s=2, tile="pt4", comm_cus=32)),
}
# phases whose check needs the candidates' CU pressure: the RCCL-fed gated GEMM must fill every
# CU it may take (a grid of num_cus - reserve) while RCCL runs beside it, or a collective that
# cannot get the CUs it needs would pass here and hang in the bench (profiles/r04/r4_33_*)
# (m = 512 d q: whole 256-row blocks per rank and stage at s = 2, >= 256 tiles of 256x256)
PRIMITIVE_SHAPES = {ph: (lambda d: (512 * d * -(-128 // d), 256, 128 * d))
                    for ph in ("rccl_fused", "rccl_fused_cm")}
PATTERN_BYTES = 1 << 20      # per rank and phase: 1 MiB (several xGMI packets, small enough)
RS_COUNT = 4096              # f32 elements per rank of the reduce-scatter check


def primitive_shape(d: int):
    """(m, n, k) of the primitive phases: whole 256-row stage blocks for every rank and stage (the
    persistent gated 256x256 kernel), k divisible by d (tp_rowwise) in whole pairs of 128-byte
    K-tiles of bf16."""
    return 512 * d, 256, 128 * d


def run_primitive_check(comm, phase: str, epochs: int = 2) -> None:
    """One primitive phase: build the real plan, run ``epochs`` times, validate the last output
    (the reference's rule) and the device spins' health."""
    import torch

    from ddlb_amd.primitives.registry import resolve

    prim, opts = PRIMITIVE_PHASES[phase]
    m, n, k = PRIMITIVE_SHAPES.get(phase, primitive_shape)(comm.world_size)
    cls, o, _ = resolve(prim, "native", dict(opts))
    impl = cls(m=m, n=n, k=k, dtype="bfloat16", **o)
    try:
        for _ in range(epochs):
            out = impl.run()
        torch.cuda.synchronize(comm.device)
        impl.check_health()
        impl.validate(out)
        comm.barrier()
    finally:
        impl.close()


def pattern(owner: int, nbytes: int, epoch: int = 1):
    """int32 words that differ per owner, epoch and position (no two ranks agree anywhere)."""
    import torch

    idx = torch.arange(nbytes // 4, dtype=torch.int64)
    v = (idx * 2654435761 + (owner + 1) * 40503 + epoch * 7919) & 0x7FFFFFFF
    return v.to(torch.int32)


def _flags(plan: Plan, d: int) -> Dict[str, Callable[..., Ref]]:
    plan.buffer("flags", max(256, 4 * 3 * d), symmetric=True, zero=True)

    def slot(base: int) -> Callable[..., Ref]:
        return lambda i, owner=None: Ref("flags", 4 * (base * d + i), owner)

    return {"READY": slot(0), "ACK": slot(1), "DONE": slot(2)}


def build_ipc_plan(rank: int, d: int, phase: str, nbytes: int = PATTERN_BYTES) -> Plan:
    """Plan of one IPC check. Buffers: ``X`` (symmetric, my pattern), ``R`` (receive region,
    ``d`` slots of ``nbytes``; symmetric for the push check)."""
    if phase not in IPC_PHASES:
        raise ValueError(f"unknown IPC preflight phase {phase}")
    peers = [p for p in range(d) if p != rank]
    plan = Plan(rank, d, nstreams=2 + max(d - 1, 1), stream_priority=[0] * (2 + max(d - 1, 1)))
    plan.meta.update(preflight=phase)
    f = _flags(plan, d)
    X = plan.buffer("X", nbytes, symmetric=True)
    R = plan.buffer("R", d * nbytes, symmetric=(phase == "ipc_push"))
    sig = SIG_KERNEL if phase == "ipc_ksig" else SIG_STREAM
    plan.signal(0, [f["READY"](rank, owner=p) for p in peers], method=sig)
    plan.wait_signal(0, [f["READY"](p) for p in peers], method=sig)
    if phase == "ipc_kernel":
        segs = [(R + p * nbytes, X.at(p), nbytes) for p in peers]
        for i in range(0, len(segs), 8):
            plan.copy_multi(0, segs[i:i + 8], max_blocks=64)
    elif phase == "ipc_sdma":
        evs = []
        for idx, p in enumerate(peers):
            st = 2 + idx
            plan.edge(0, st)
            plan.copy(st, R + p * nbytes, X.at(p), nbytes, method=COPY_ENGINE)
            e = plan.event()
            plan.record(st, e)
            evs.append(e)
        for e in evs:
            plan.wait(0, e)
    elif phase == "ipc_batch":
        segs = [(R + p * nbytes, X.at(p), nbytes) for p in peers]
        for i in range(0, len(segs), 8):
            plan.copy_batch(0, segs[i:i + 8])
    elif phase == "ipc_push":
        for idx, p in enumerate(peers):
            st = 2 + idx
            plan.edge(0, st)
            plan.copy(st, (R + rank * nbytes).at(p), X, nbytes, method=COPY_ENGINE)
            plan.signal(st, [f["DONE"](rank, owner=p)], method=SIG_STREAM)
        plan.wait_signal(0, [f["DONE"](p) for p in peers], method=SIG_STREAM)
    # nobody's X / R is touched again (next epoch's fill, teardown) before every peer is done
    plan.signal(0, [f["ACK"](rank, owner=p) for p in peers], method=sig)
    plan.wait_signal(0, [f["ACK"](p) for p in peers], method=sig)
    return plan


def build_rccl_plan(rank: int, d: int, nbytes: int = PATTERN_BYTES,
                    count: int = RS_COUNT) -> Plan:
    """All-gather of ``SEND`` (bytes) into ``AG`` and an f32 reduce-scatter ``RSIN`` -> ``RSOUT``
    on our own communicator, on a side stream (as the pipelines enqueue them)."""
    plan = Plan(rank, d, nstreams=2, stream_priority=[0, 1])
    plan.meta.update(preflight="rccl")
    send = plan.buffer("SEND", nbytes)
    ag = plan.buffer("AG", d * nbytes)
    rsin = plan.buffer("RSIN", d * count * 4)
    rsout = plan.buffer("RSOUT", count * 4)
    plan.edge(0, 1)
    plan.allgather(1, send, ag, nbytes, DT_U8)
    plan.reduce_scatter(1, rsin, rsout, count, DT_F32)
    plan.edge(1, 0)
    return plan


def rs_input(owner: int, d: int, count: int = RS_COUNT):
    """Reduce-scatter input of ``owner``: small integers, so every f32 sum is exact."""
    import torch

    idx = torch.arange(d * count, dtype=torch.int64)
    return ((idx % 13) + 1 + owner * 3).to(torch.float32)


def rs_expected(rank: int, d: int, count: int = RS_COUNT):
    import torch

    return sum(rs_input(q, d, count) for q in range(d))[rank * count:(rank + 1) * count].to(
        torch.float32)


# ------------------------------------------------------------------------------ execution
class _Progress:
    """Per-phase results, rewritten to ``path`` after every phase (a hang leaves the rest out)."""

    def __init__(self, path: Optional[str]):
        self.path = path
        self.res: Dict[str, str] = {}

    def put(self, phase: str, status: str) -> None:
        self.res[phase] = status
        if self.path:
            tmp = self.path + ".tmp"
            with open(tmp, "w") as fh:
                json.dump(self.res, fh)
            os.replace(tmp, self.path)


def _run_checked(name: str, progress: _Progress, fn: Callable[[], None]) -> bool:
    t0 = time.perf_counter()
    try:
        detail = fn()
    except Exception as e:  # recorded, never raised: the other phases still run
        progress.put(name, f"failed: {type(e).__name__}: {str(e).splitlines()[0][:200]}"
                     if str(e) else f"failed: {type(e).__name__}")
        return False
    extra = f"; {detail}" if isinstance(detail, str) and detail else ""
    progress.put(name, f"ok ({(time.perf_counter() - t0) * 1e3:.0f} ms{extra})")
    return True


def _check_eq(got, want, what: str) -> None:
    import torch

    if not torch.equal(got.cpu(), want.cpu()):
        bad = int((got.cpu() != want.cpu()).sum())
        raise AssertionError(f"{what}: {bad} of {want.numel()} words differ")


def _ipc_phase(comm, phase: str, nbytes: int, epochs: int) -> Callable[[], None]:
    """The check of one IPC phase (a data-movement plan on the native executor)."""
    import torch

    def one():
        ctx = comm.native()
        r, d, dev = comm.rank, comm.world_size, comm.device
        plan = build_ipc_plan(r, d, phase, nbytes)
        bound = ctx.bind(plan)
        try:
            for ep in range(1, epochs + 1):
                x = bound.buffer("X").view(torch.int32)
                x.copy_(pattern(r, nbytes, ep).to(dev))
                bound.buffer("R").view(torch.int32).fill_(-1)
                torch.cuda.synchronize(dev)
                comm.barrier()  # every rank's X of this epoch is in place
                bound.run()
                torch.cuda.synchronize(dev)
                bound.check_health()
                if phase == "ipc_batch":
                    status = ctx.C.copy_batch_status()
                    if not status.startswith(("hipMemcpyBatchAsync", "hipGraph")):
                        raise RuntimeError(f"batched copies: {status}")
                if phase in ("ipc_kernel", "ipc_sdma", "ipc_push", "ipc_batch"):
                    rv = bound.buffer("R").view(torch.int32)
                    for p in range(d):
                        if p != r:
                            _check_eq(rv[p * nbytes // 4:(p + 1) * nbytes // 4],
                                      pattern(p, nbytes, ep), f"{phase} slot of rank {p}")
                comm.barrier()  # nobody refills X while a peer may still read it
        finally:
            bound.close()

    return one


def phase_checks(comm, family: str, nbytes: int = PATTERN_BYTES, count: int = RS_COUNT,
                 epochs: int = 2) -> Dict[str, Callable[[], None]]:
    """phase -> check for one family (``rccl`` | ``ipc``): every declared phase has exactly one
    check here (``tests/test_preflight.py`` asserts it), so a phase missing from a progress file
    can only mean that its child was killed mid-phase (a timeout), never an unimplemented phase."""
    fns: Dict[str, Callable[[], None]] = {}
    phases = RCCL_PHASES if family == "rccl" else IPC_PHASES
    for ph in phases:
        if ph in PRIMITIVE_PHASES:
            fns[ph] = (lambda ph=ph: run_primitive_check(comm, ph, epochs))
        elif family == "ipc":
            fns[ph] = _ipc_phase(comm, ph, nbytes, epochs)
    if family == "rccl":
        fns["torch_nccl"] = lambda: _torch_nccl_check(comm)
        fns["rccl"] = lambda: _own_rccl_check(comm, nbytes, count)
        fns["rccl_cap"] = lambda: _rccl_cap_check(comm)
    return fns


def _run_family(comm, family: str, phases, progress_path, **kw) -> Dict[str, str]:
    prog = _Progress(progress_path)
    fns = phase_checks(comm, family, **kw)
    for ph in phases:
        fn = fns.get(ph)
        if fn is None:  # (a caller asking for a phase of the other family)
            prog.put(ph, "failed: no such preflight check")
            continue
        _run_checked(ph, prog, fn)
    return prog.res


def run_ipc_checks(comm, phases=IPC_PHASES, progress_path: Optional[str] = None,
                   nbytes: int = PATTERN_BYTES, epochs: int = 2) -> Dict[str, str]:
    return _run_family(comm, "ipc", phases, progress_path, nbytes=nbytes, epochs=epochs)


def _torch_nccl_check(comm) -> None:
    """torch's RCCL process group: a SUM all-reduce of rank-dependent values."""
    import torch
    import torch.distributed as dist

    r, d, dev = comm.rank, comm.world_size, comm.device
    if dist.get_backend() == "nccl":
        grp = None
    else:  # control plane forced to gloo: build a separate RCCL group
        grp = dist.new_group(backend="nccl")
    t = torch.full((1024,), float(r + 1), device=dev)
    dist.all_reduce(t, group=grp)
    torch.cuda.synchronize(dev)
    want = torch.full((1024,), float(d * (d + 1) // 2))
    _check_eq(t, want, "all_reduce")
    if grp is not None:
        dist.destroy_process_group(grp)


def _own_rccl_check(comm, nbytes: int, count: int) -> None:
    """Our own communicator on our streams: all-gather + reduce-scatter, two epochs."""
    import torch

    r, d, dev = comm.rank, comm.world_size, comm.device
    ctx = comm.native()
    bound = ctx.bind(build_rccl_plan(r, d, nbytes, count))
    try:
        for ep in (1, 2):
            bound.buffer("SEND").view(torch.int32).copy_(pattern(r, nbytes, ep).to(dev))
            bound.buffer("RSIN").view(torch.float32).copy_(rs_input(r, d, count).to(dev))
            torch.cuda.synchronize(dev)
            bound.run()
            torch.cuda.synchronize(dev)
            ag = bound.buffer("AG").view(torch.int32)
            for q in range(d):
                _check_eq(ag[q * nbytes // 4:(q + 1) * nbytes // 4],
                          pattern(q, nbytes, ep), f"all-gather slot of rank {q}")
            _check_eq(bound.buffer("RSOUT").view(torch.float32)[:count],
                      rs_expected(r, d, count), "reduce-scatter")
            comm.barrier()
    finally:
        bound.close()


def fused_rccl_cap(d: int) -> int:
    """The CTA cap the RCCL-fed fused candidates bind their communicator with (the plan's
    ``rccl_max_ctas``, ``NativeContext.rccl``), from the rccl_fused phase's own plan (built for
    at least 2 ranks: at world 1 nothing is gated and the plan carries no cap)."""
    d = max(int(d), 2)
    from ddlb_amd.parallel.algorithms import build_tp_columnwise
    from ddlb_amd.parallel.context import rccl_gate_cap
    from ddlb_amd.parallel.plan import DT_BF16
    from ddlb_amd.primitives.native_common import algo_config
    from ddlb_amd.primitives.registry import resolve

    prim, opts = PRIMITIVE_PHASES["rccl_fused"]
    cls, o, _ = resolve(prim, "native", dict(opts))
    merged = {**cls.DEFAULT_OPTIONS, **o}
    for key, alias in cls.OPTION_ALIASES.items():
        merged[key] = alias.get(merged[key], merged[key])
    plan, _ = build_tp_columnwise(0, d, *PRIMITIVE_SHAPES["rccl_fused"](d), DT_BF16, DT_BF16,
                                  algo_config(merged))
    return rccl_gate_cap(plan)


def cap_probe(holder, launch, done, barrier, ncu: int, cap: int, resident_s: float = 2.0,
              finish_s: float = 5.0, sleep=time.sleep, clock=time.perf_counter) -> Dict:
    """The rccl_cap observation, independent of the device layer (tests drive it with fakes):
    hold ``ncu - cap`` CUs (``holder.start(n)``; wait until ``holder.arrived() == n``), barrier,
    ``launch()`` the capped collective, poll ``done()`` for ``finish_s``, release the holders in
    every case. Raises if the holders never became resident, if the collective did not finish
    while they held their CUs, or if a holder's own bounded spin gave up."""
    n = ncu - cap
    if n < 1:
        raise ValueError(f"cap {cap} leaves nothing to hold on {ncu} CUs")
    holder.start(n)
    try:
        t0 = clock()
        while holder.arrived() < n and clock() - t0 < resident_s:
            sleep(0.001)
        got = holder.arrived()
        if got < n:
            raise RuntimeError(f"only {got} of {n} holder workgroups became resident in "
                               f"{resident_s:.0f} s (another process on the GPU?)")
        barrier()  # every rank holds its CUs before any collective starts
        t1 = clock()
        launch()
        while not done() and clock() - t1 < finish_s:
            sleep(0.0002)
        held_ms = (clock() - t1) * 1e3
        finished = done()
    finally:
        holder.release()
    if holder.timeout_bits():
        raise RuntimeError("a holder's bounded spin gave up (host release lost?)")
    if not finished:
        raise RuntimeError(f"the all-gather capped at {cap} workgroups did not finish within "
                           f"{finish_s:.0f} s beside {n} held CUs: RCCL needs more CUs than the "
                           "cap (or other ones) -- the RCCL-fed gated GEMM could hang here")
    return {"held_cus": n, "cap": cap, "held_ms": round(held_ms, 3)}


def _rccl_cap_check(comm, nbytes: int = PATTERN_BYTES) -> str:
    """rccl_cap on the device: the capped all-gather beside ``num_cus - cap`` held CUs, checked
    bytewise, and timed against the same all-gather with nothing held."""
    import torch

    from ddlb_amd.parallel.plan import DT_U8

    r, d, dev = comm.rank, comm.world_size, comm.device
    ctx = comm.native()
    cap = fused_rccl_cap(d)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    rc = ctx.rccl(cap)
    send = pattern(r, nbytes).to(dev)
    recv = torch.full((d * nbytes // 4,), -1, dtype=torch.int32, device=dev)
    s_comm = torch.cuda.Stream(dev, priority=-1)
    s_hold = torch.cuda.Stream(dev)
    ev = torch.cuda.Event()

    def launch():
        rc.all_gather(send.data_ptr(), recv.data_ptr(), nbytes, DT_U8, s_comm.cuda_stream)
        ev.record(s_comm)

    torch.cuda.synchronize(dev)
    comm.barrier()
    t0 = time.perf_counter()
    launch()
    ev.synchronize()
    free_ms = (time.perf_counter() - t0) * 1e3
    recv.fill_(-1)
    torch.cuda.synchronize(dev)
    holder = ctx.C.CuHolder(comm.device.index)
    # (the barrier inside the hold must not sync the device: the holders spin until released)
    res = cap_probe(_Holder(holder, s_hold.cuda_stream), launch, ev.query,
                    lambda: comm.host_barrier("cap"), ncu, cap)
    torch.cuda.synchronize(dev)
    for q in range(d):
        _check_eq(recv[q * nbytes // 4:(q + 1) * nbytes // 4], pattern(q, nbytes),
                  f"capped all-gather slot of rank {q}")
    comm.barrier()
    return (f"cap {cap}: all-gather finished in {res['held_ms']:.2f} ms beside {res['held_cus']} "
            f"held CUs (free {free_ms:.2f} ms)")


class _Holder:
    """``cap_probe``'s holder interface over the native ``CuHolder``."""

    def __init__(self, native, stream: int):
        self.h, self.stream = native, stream

    def start(self, n: int) -> None:
        self.h.start(n, self.stream)

    def arrived(self) -> int:
        return int(self.h.arrived())

    def release(self) -> None:
        self.h.release()

    def timeout_bits(self) -> int:
        return int(self.h.timeout_bits())


def run_rccl_checks(comm, phases=RCCL_PHASES, progress_path: Optional[str] = None,
                    nbytes: int = PATTERN_BYTES, count: int = RS_COUNT) -> Dict[str, str]:
    """Every RCCL phase, in ``RCCL_PHASES`` order: torch's group, our communicator, the RCCL-fed
    gated GEMM and its CU-split form (``rccl_fused_cm``: a plain fused hang must not drop it)."""
    return _run_family(comm, "rccl", phases, progress_path, nbytes=nbytes, count=count)


def families_ok(results: Dict[str, str]) -> Dict[str, bool]:
    """Which data-plane families a benchmark may use, from merged (all-rank) phase results."""
    ok = {k: str(v).startswith("ok") for k, v in results.items()}
    return ok


def needs(impl: str, opts: Dict, primitive: str = "tp_columnwise") -> List[str]:
    """Preflight checks a benchmark candidate relies on (``bench.py`` drops it if any failed)."""
    if impl == "pytorch":
        return ["torch_nccl"]
    if impl != "native":
        return []
    backend = opts.get("backend", "rccl")
    alg = opts.get("algorithm", "default")
    fused = bool(opts.get("fused", False))
    if backend in ("rccl", "nccl"):
        if not fused:
            return ["rccl"]
        if int(opts.get("comm_cus", 0)) > 0:  # a CU split: RCCL has CUs of its own, no cap
            return ["rccl", "rccl_fused_cm"]
        return ["rccl", "rccl_cap", "rccl_fused"]
    out = ["ipc"]
    # a missing "graph" key is the option default "auto" (graph replay whenever capturable, and
    # graph mode always signals with the kernels); the rowwise IPC plans send READY with the
    # signal kernel whatever ``signal`` says
    if (opts.get("graph", "auto") in (True, "auto", "true") or opts.get("signal") == "kernel"
            or primitive == "tp_rowwise"):
        out.append("ipc_ksig")
    proto = opts.get("multicast_protocol", "memcpy")
    if alg == "direct" or proto == "kernel":
        out.append("ipc_kernel")   # peer HBM read by CUs (copy kernel, in-kernel AG, LDS-DMA)
    elif proto == "batch_memcpy":
        out.append("ipc_batch")
    elif opts.get("direction") == "push":
        out.append("ipc_push")
    else:
        out.append("ipc_sdma")
    if primitive == "tp_columnwise" and fused and alg == "coll_pipeline" and proto == "kernel":
        out.append("ipc_agk")
    if primitive == "tp_rowwise" and fused and alg == "p2p_pipeline":
        out.append("ipc_dstore")
    return out


def merge(per_rank: List[Dict[str, str]], phases) -> Dict[str, str]:
    """One status per phase over every rank: ok only if every rank passed it; a phase missing on
    some rank (its child was killed mid-phase) is a timeout."""
    out: Dict[str, str] = {}
    for ph in phases:
        st = [res.get(ph) for res in per_rank]
        bad = [s for s in st if s is not None and not str(s).startswith("ok")]
        if bad:
            out[ph] = str(bad[0])
        elif any(s is None for s in st):
            out[ph] = "failed: timeout"
        else:
            out[ph] = st[0]
    return out
