#!/usr/bin/env python3
"""Flagship benchmark: tp_columnwise AG+GEMM, m=65536 (sequence), n=1024, k=1024, bf16.

BASELINE.json metric: "ms/iter + effective TFLOP/s, tp_columnwise AG+GEMM m=65536 bf16 at
1/2/4/8 GPUs". n=k=1024 is the reference README's m=65536 example (``README.md:37-39``).

Contract (driver):  python bench.py --gpus N --steps K --warmup W
  * N>1 is launched by torch.distributed.run, one rank per GPU (RANK/LOCAL_RANK/WORLD_SIZE env);
    started without a launcher, ``--gpus N`` runs torch.distributed.run itself as a child
    process and relays rank 0's line (``self_launch``);
  * W untimed warmups, then EXACTLY K timed steps bracketed by barrier + device sync on both
    sides; ms_per_step is the MAX over ranks;
  * rank 0 prints ONE JSON line. ``value`` = whole-job effective TFLOP/s = N * 2*m*n*k / t
    (every rank computes the full [m,k]x[k,n] on its own N-slice of the weight: weak scaling in
    N); ``per_gpu_tflops`` is the reference harness's per-GPU number (``ddlb/benchmark.py:211``).

Other BASELINE configs through the same machinery: ``--primitive tp_rowwise -m 16384 -n 8192
-k 8192`` (config #3, GEMM + reduce-scatter; strong scaling: the harness number is the whole-job
aggregate) and ``--dtype float8_e4m3fn`` (config #5; adds the block-scaled MX-fp8 candidates).

What runs in the timed region: only the ``native`` slot's own hand-written MFMA kernels (with
RCCL / IPC data movement at N>1). The vendor library (hipBLASLt through ``torch.matmul``, RCCL
through torch) is measured beside it as the ``pytorch`` / ``compute_only(torch)`` slots and
reported as ``vendor_ms``; it becomes the headline only if every native candidate fails, and
the JSON then says so (``implementation``, ``gemm``).

Process model (robust by construction): the launched processes never touch the GPU. They form
a gloo group and run every measurement in a child process per rank (fresh HIP context, its own
rendezvous port, a hard timeout). At N>1 a preflight (``ddlb_amd.parallel.preflight``) first
checks, in time-limited children, that RCCL and the IPC / xGMI mechanisms work across this
node's GPUs; candidate families that fail are dropped, and a broken RCCL control plane makes
the children coordinate over gloo instead. An autotuner then times each candidate (validated,
MAX over ranks) in the order of the one-GPU per-rank budget (``scripts/plan_budget.py``), and
the winner runs the timed measurement (falling back
to the next fastest if it fails there). The whole job runs against ONE wall-clock deadline
(``--deadline-s``): tuning stops early enough to leave the final run its time, and every child's
timeout is cut to what is left, so a node where candidates hang still reports inside it.
Every rank issues the same number of run() calls (the pre-warm count is MAX-reduced), as each
call holds collectives / epoch-matched signals. Synthetic U[-1,1) inputs of the named shape (no
datasets exist offline); the result is validated against an fp32 reference, with the
reference's rule (atol = 1e-3 k) and a tight internal bound (max|err| <= 2^-7 max|ref| + k 2^-12).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

TIMING = ("cpu_clock window: barrier + device sync, K back-to-back run() calls, device sync; "
          "mean per step, MAX over ranks")

_COLL4 = dict(algorithm="coll_pipeline", backend="rccl", s=4)
_DEF = dict(algorithm="default", backend="rccl")
_P2P = dict(algorithm="p2p_pipeline", backend="ipc", multicast_protocol="memcpy")
_COLL_IPC = dict(algorithm="coll_pipeline", backend="ipc", multicast_protocol="memcpy", s=4)
_DEF_K = dict(algorithm="default", backend="ipc", multicast_protocol="kernel", copy_blocks=128)
# In-kernel all-gather ("agk"): ONE launch per run; its first copy_blocks workgroups pull the
# peers' row blocks over xGMI and flag them, the rest run the persistent GEMM gated on the flags
# (no copy streams, no host op per block, one kernel to capture).
_AGK = dict(algorithm="coll_pipeline", backend="ipc", multicast_protocol="kernel", fused=True,
            s=8, copy_blocks=32)


def _graph(opts):
    return dict(opts, graph=True)


# N > 1 pool. Order: the forms that cannot hang by construction first (direct/ipc: one ungated
# GEMM reading the peers' shards in place; the in-kernel all-gather: a gated GEMM fed only by its
# own launch's copy workgroups), then the RCCL-fed gated GEMMs (their communicator capped at the
# GEMM's CU reserve, so a collective always fits beside the spinning tiles) and the plain RCCL
# pipelines, interleaved with the next IPC forms; within a family, the one-GPU per-rank budget's
# order (scripts/plan_budget.py --world 8, profiles/r04/r4_6_budget_col8.txt: rank 0's d = 8 plan
# replayed on one GPU, transfers as local copies -- an emulated lower bound that cannot see the
# links, so it never outranks the no-hang forms). The preflight (RCCL, IPC, in-kernel all-gather,
# direct store, RCCL-fed gated GEMM, across the real peers) drops whatever this node cannot run.
# Sized so that every candidate plus two hangs fits the tuning budget (tests/test_bench_cpu.py
# test_pool_fits_tuning_budget): dominated and host-bound forms live in CANDIDATES_EXTRA.
# "/graph": the whole plan is captured once and replayed with one hipGraphLaunch per run (the IPC
# pipelines issue ~200 HIP calls per run at d = 8 otherwise, profiles/r02/r2_13_*).
CANDIDATES = [
    # one GEMM reading every peer's shard in place over xGMI (pt4 through a shard table)
    ("direct/ipc", "native", dict(algorithm="direct", backend="ipc")),
    # in-kernel all-gather: budget 0.128 ms (graph), GEMM work 0.085 ms
    ("coll_pipeline/ipc/agk32/s4/graph", "native", _graph(dict(_AGK, s=4))),
    # RCCL stage all-gathers feeding ONE flag-gated persistent GEMM over all m rows (the
    # flagship's 1024-tile pt4 kernel at m = 65536; per stage a signal kernel raises the
    # arrival flags, the own rows run first, ungated): no under-filled stage GEMMs (at d = 8,
    # s = 8 a stage GEMM has 128 tiles of 256^2 for 256 CUs). Budget 0.196 ms (s4), GEMM work
    # 0.116-0.119 ms (5 tile rounds on the CUs RCCL leaves); RCCL capped at 32 workgroups
    ("coll_pipeline/rccl/s4/fused", "native", dict(_COLL4, fused=True)),
    ("coll_pipeline/rccl/s4", "native", _COLL4),
    ("default/rccl", "native", _DEF),
    ("p2p_pipeline/rccl/fused", "native", dict(algorithm="p2p_pipeline", backend="rccl",
                                               fused=True)),
    ("coll_pipeline/ipc/agk32/s8/graph", "native", _graph(_AGK)),
    ("coll_pipeline/rccl/s8/fused", "native", dict(_COLL4, s=8, fused=True)),
    ("default/ipc/kernel", "native", _DEF_K),
    ("coll_pipeline/rccl/s8", "native", dict(_COLL4, s=8)),
    ("p2p_pipeline/rccl", "native", dict(algorithm="p2p_pipeline", backend="rccl")),
    ("default/ipc/push", "native", dict(_P2P, algorithm="default", direction="push")),
    ("coll_pipeline/ipc/agk64/s8/graph", "native", _graph(dict(_AGK, copy_blocks=64))),
    ("p2p_pipeline/ipc/memcpy/graph", "native", _graph(_P2P)),
    ("coll_pipeline/ipc/memcpy/s4/graph", "native", _graph(_COLL_IPC)),
    # the stage GEMMs next to RCCL's CU-resident kernels: 128x128 tiles (4x as many, dispatched
    # dynamically) let the CUs busy with RCCL simply take fewer of them
    ("coll_pipeline/rccl/s4/128/c16", "native", dict(_COLL4, tile="128x128",
                                                      _env={"NCCL_MAX_NCHANNELS": "16"})),
    ("coll_pipeline/ipc/kernel/s4", "native", dict(_COLL_IPC, multicast_protocol="kernel",
                                                   copy_blocks=128, tile="128x128")),
    # the RCCL-fed fused GEMM on a CU split (RCCL on 32 CUs of its own, the gated GEMM on the
    # other 224): immune to a collective starved by the spinning tiles, but the masked GEMM runs
    # 1.5x slower (emulated 0.302 vs 0.181 ms, profiles/r04/r4_36_*): a fallback, with its own
    # preflight phase so a plain fused hang does not drop it. CU-masked streams carry no priority
    # (HIP's hipExtStreamCreateWithCUMask takes none): its comm stream runs at normal priority,
    # which a CU split does not need (test_rccl_data_plane_world1 asserts what HIP gives)
    ("coll_pipeline/rccl/s4/fused/cumask", "native", dict(_COLL4, fused=True, comm_cus=32)),
]
# Measured but dominated at d = 8, or host-bound: not in the default pool (each costs tuning
# time on the 8-GPU node), still selectable with --candidates / --algorithm. Host cost per run
# (eager) and the emulated plan time from profiles/r04/r4_6_budget_col8.txt:
CANDIDATES_EXTRA = [
    ("coll_pipeline/rccl/s4/128", "native", dict(_COLL4, tile="128x128")),   # 0.263 ms
    ("coll_pipeline/ipc/kernel/s8/graph", "native", _graph(dict(             # 0.330 ms graph
        _COLL_IPC, s=8, multicast_protocol="kernel", copy_blocks=128, tile="128x128"))),
    ("coll_pipeline/ipc/push/s4", "native", dict(_COLL_IPC, direction="push")),  # host 411 us
    # batch_memcpy: without hipMemcpyBatchAsync (torch's HIP 7.0 runtime) an eager batch runs as
    # one launch of a graph of memcpy nodes (the ipc_batch phase passes with it); kept out of the
    # default pool for its cost: the s8 graph form's budget is dominated by the RCCL / agk forms
    ("coll_pipeline/ipc/batch/s8/graph", "native", _graph(dict(
        _COLL_IPC, s=8, multicast_protocol="batch_memcpy"))),
    ("coll_pipeline/ipc/memcpy/s8/graph", "native", _graph(dict(_COLL_IPC, s=8))),  # 0.779 ms
    # one flag-gated GEMM fed by copy-engine pulls: eager only (a graph would have to order the
    # gated GEMM after every copy stream, see PlanExecutor::graph_capturable); host 682 us
    ("coll_pipeline/ipc/memcpy/s8/fused", "native", dict(_COLL_IPC, s=8, fused=True)),
    # RCCL's kernels on a CU-masked comm stream (csrc/comm: hipExtStreamCreateWithCUMask), the
    # stage GEMMs sized to the complement (the masked GEMMs lose 32-64 CUs for the whole run:
    # 0.73-1.51 ms emulated)
    ("coll_pipeline/rccl/s4/cumask", "native", dict(_COLL4, comm_cus=32, register=True)),
    ("coll_pipeline/rccl/s8/cumask", "native", dict(_COLL4, s=8, comm_cus=32, register=True)),
    ("coll_pipeline/rccl/s4/cumask64", "native", dict(_COLL4, comm_cus=64)),
    ("p2p_pipeline/ipc/memcpy/cs2", "native", dict(_P2P, copy_streams=2)),        # host 337 us
    # each peer's chunks split over 2 copy streams (2 copy engines per link): 1.17 ms graph
    ("coll_pipeline/ipc/memcpy/s8/cs2/graph", "native",
     dict(_COLL_IPC, s=8, copy_streams=2, graph=True)),
    ("coll_pipeline/ipc/memcpy/s8", "native", dict(_COLL_IPC, s=8)),             # host 562 us
]
VENDOR = [
    ("pytorch(rccl+hipblaslt)", "pytorch", dict(backend="nccl", empty_cache=False)),
]
# world 1: the all-gather is the identity; the plan is one GEMM (our kernel families)
WORLD1 = [
    ("gemm (world=1)/auto", "native", _DEF),
    ("gemm (world=1)/t4", "native", dict(_DEF, tile="t4")),
    ("gemm (world=1)/pt8", "native", dict(_DEF, tile="pt8")),
]
WORLD1_VENDOR = [
    ("compute_only(hipblaslt)", "compute_only", dict(size="unsharded", gemm="torch")),
    # F.linear on the [n, k] weight: hipBLASLt's fastest layout, the like-for-like comparison
    ("compute_only(hipblaslt,nt)", "compute_only", dict(size="unsharded", gemm="torch_nt")),
    ("pytorch(rccl+hipblaslt)", "pytorch", dict(backend="nccl", empty_cache=False)),
]
# tp_rowwise (GEMM + sequence-parallel reduce-scatter; BASELINE config #3)
_RK = dict(backend="ipc", multicast_protocol="kernel", copy_blocks=128)
ROW_CANDIDATES = [
    ("row/default/rccl", "native", dict(algorithm="default", backend="rccl")),
    ("row/coll_pipeline/rccl/s4", "native", dict(algorithm="coll_pipeline", backend="rccl", s=4)),
    ("row/coll_pipeline/rccl/s4/128", "native", dict(algorithm="coll_pipeline", backend="rccl",
                                                     s=4, tile="128x128")),
    ("row/p2p_pipeline/rccl", "native", dict(algorithm="p2p_pipeline", backend="rccl")),
    # direct store: ONE GEMM whose epilogue writes every peer's partial into its receive slot
    # over xGMI (shard-interleaved tiles: all links at once), then one local d-way reduce
    ("row/p2p_pipeline/ipc/direct/graph", "native", _graph(dict(algorithm="p2p_pipeline",
                                                                backend="ipc", fused=True))),
    ("row/p2p_pipeline/ipc/direct", "native", dict(algorithm="p2p_pipeline", backend="ipc",
                                                   fused=True)),
    ("row/default/ipc/kernel", "native", dict(_RK, algorithm="default")),
    ("row/coll_pipeline/ipc/kernel/s4", "native", dict(_RK, algorithm="coll_pipeline", s=4)),
    ("row/p2p_pipeline/ipc/memcpy", "native", dict(algorithm="p2p_pipeline", backend="ipc")),
    ("row/coll_pipeline/ipc/kernel/s4/graph", "native", _graph(dict(_RK, algorithm="coll_pipeline",
                                                                    s=4))),
    ("row/p2p_pipeline/ipc/memcpy/graph", "native", _graph(dict(algorithm="p2p_pipeline",
                                                                 backend="ipc"))),
]
ROW_VENDOR = [
    ("row/pytorch(rccl+hipblaslt)", "pytorch", dict(backend="nccl", empty_cache=False)),
]
ROW_WORLD1 = [
    ("row/gemm (world=1)/auto", "native", dict(algorithm="default", backend="rccl")),
    ("row/gemm (world=1)/t4", "native", dict(algorithm="default", backend="rccl", tile="t4")),
]
ROW_WORLD1_VENDOR = [
    ("row/compute_only(hipblaslt)", "compute_only", dict(gemm="torch")),
    ("row/compute_only(hipblaslt,nt)", "compute_only", dict(gemm="torch_nt")),
    ("row/pytorch(rccl+hipblaslt)", "pytorch", dict(backend="nccl", empty_cache=False)),
]


FP8_NON_MX = 3  # N > 1 fp8: non-scaled fp8 (the bf16 MFMA rate) kept for the first few forms only


def candidate_pool(primitive: str, dtype: str, world: int, extra: bool = False):
    """(label, impl, options) list for one primitive / dtype / world size: our native
    candidates first, then the vendor-library slots (measured for ``vendor_ms``). fp8 inputs add
    the block-scaled MX-fp8 MFMA (2x the bf16 rate) to every native candidate; at N > 1 the
    non-scaled fp8 forms (the bf16 rate) are kept for the first ``FP8_NON_MX`` only, so the pool
    stays inside the tuning budget. ``extra``: also the dominated forms (``CANDIDATES_EXTRA``)."""
    row = primitive == "tp_rowwise"
    if world == 1:
        native, vendor = (ROW_WORLD1, ROW_WORLD1_VENDOR) if row else (WORLD1, WORLD1_VENDOR)
    else:
        native, vendor = (ROW_CANDIDATES, ROW_VENDOR) if row else (CANDIDATES, VENDOR)
        if extra and not row:
            native = native + CANDIDATES_EXTRA
    if dtype == "float8_e4m3fn":
        mx = [(lbl + "/mx", impl, dict(opts, gemm_mode="mx")) for lbl, impl, opts in native]
        if world == 1 or extra:
            native = native + mx
        else:  # MX first: twice the MFMA rate of every non-scaled form
            native = mx + native[:FP8_NON_MX]
        vendor = [c for c in vendor if c[1] != "compute_only"]  # torch.matmul has no fp8
    return list(native) + list(vendor)


# ------------------------------------------------------------------------------- child
def prewarm_runs(impl, comm, prewarm_ms: float, calib: int = 4) -> int:
    """Number of extra pre-warm run() calls after a ``calib``-call calibration batch, agreed by
    all ranks (MAX over ranks) so every rank issues the same sequence of collectives."""
    import torch

    if prewarm_ms <= 0:
        return 0
    comm.synchronize()
    t0 = time.perf_counter()
    for _ in range(calib):
        impl.run()
    comm.synchronize()
    per_ms = max((time.perf_counter() - t0) * 1e3 / calib, 1e-3)
    want = torch.tensor([min(int(prewarm_ms / per_ms), 20000)], dtype=torch.float64,
                        device=comm.device)
    comm.all_reduce_max(want)
    return int(want.item())


def _check(impl, out, res) -> bool:
    """Validate one output: the reference's rule, then the tight internal bound. A mismatch is
    recorded in ``res`` (not raised)."""
    try:
        impl.validate(out)
    except AssertionError as e:
        res["validation"] = str(e).splitlines()[0][:200]
        return False
    num = impl.numerics(out)
    res["max_err"], res["err_bound"] = round(num["max_err"], 6), round(num["bound"], 6)
    if not num["ok"]:
        res["validation"] = (f"tight check: max|err| {num['max_err']:.4g} > "
                             f"{num['bound']:.4g} (2^-7 max|ref| + k 2^-12)")
        return False
    return True


def harness_times(impl, comm, iters: int):
    """The reference's default timing (``ddlb/benchmark.py:161-172``): per iteration a device
    sync + barrier, then perf_counter around run(); synchronize(). MAX over ranks per
    iteration (``:190-204``); returns the per-iteration ms."""
    import torch

    times = []
    for _ in range(iters):
        comm.barrier()
        t0 = time.perf_counter()
        impl.run()
        comm.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    t = torch.tensor(times, dtype=torch.float64, device=comm.device)
    comm.all_reduce_max(t)
    return [float(x) for x in t.cpu()]


def child_main(a) -> int:
    """One measurement on this rank's GPU; writes a JSON result file (rank 0 aggregates)."""
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.primitives.registry import resolve

    res = {"ok": False}
    try:
        comm = Communicator()
        comm.ensure_process_group(timeout_s=a.child_timeout)
        cls, opts, _ = resolve(a.primitive, a.child_impl, json.loads(a.child_opts))
        impl = cls(m=a.m, n=a.n, k=a.k, dtype=a.dtype, **opts)
        valid = None
        if a.validate:
            out = impl.run()
            comm.synchronize()
            valid = _check(impl, out, res)
        # untimed pre-warm: keep the GPU busy for ~prewarm_ms so the timed window does not
        # include the clock ramp out of idle (measured: 10 warmups of this step leave the
        # first 50 timed steps ~14 % slow). Then the W warmup steps of the contract.
        # Every rank must issue the SAME number of run() calls (each one holds collectives /
        # epoch-matched cross-rank signals), so the count is derived from a calibration batch
        # and MAX-reduced over ranks — never from each rank's own wall clock.
        for _ in range(prewarm_runs(impl, comm, a.prewarm_ms)):
            impl.run()
        comm.synchronize()
        for _ in range(a.warmup):
            impl.run()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = impl.run()
        comm.synchronize()
        t1 = time.perf_counter()
        comm.barrier()
        t = torch.tensor([(t1 - t0) * 1e3 / a.steps], dtype=torch.float64, device=comm.device)
        comm.all_reduce_max(t)
        # after the timed loop: no device-side spin may have given up (a peer that never
        # signalled leaves stale data behind a "successful" step), and the output of the LAST
        # timed step must validate too (cross-rank ordering bugs show up under back-to-back
        # epochs, not on the first, isolated run)
        impl.check_health()
        if a.validate and valid:
            valid = _check(impl, out, res)
        if a.harness_iters > 0:
            ht = harness_times(impl, comm, a.harness_iters)
            res["harness_mean_ms"] = sum(ht) / len(ht)
            impl.check_health()
        res.update(ok=True, ms=float(t.item()), valid=valid)
        if opts.get("multicast_protocol") == "batch_memcpy":
            # a batch_memcpy time is a batched submission only if the API call succeeded
            from ddlb_amd.ops import load

            res["copy_batch"] = load().copy_batch_status()
        impl.close()
        comm.destroy()
    except Exception as e:  # reported to the parent, never raised
        res["error"] = f"{type(e).__name__}: {str(e)[:300]}"
    with open(a.child_out, "w") as f:
        json.dump(res, f)
    return 0


def diagnose_child(a) -> int:
    """First-contact diagnostics of the N>1 data plane on this rank (ddlb_amd.parallel.diagnose):
    xGMI pull bandwidth per peer, RCCL bus bandwidth on the default and the capped communicator,
    and a per-op timeline of the winner (built eagerly). Written to --child-out; never raises."""
    res = {}
    try:
        from ddlb_amd.communicator import Communicator
        from ddlb_amd.parallel import diagnose
        from ddlb_amd.primitives.registry import resolve

        comm = Communicator()
        comm.ensure_process_group(timeout_s=min(a.child_timeout, 60.0))
        spec = json.loads(a.child_opts)
        esz = 1 if a.dtype == "float8_e4m3fn" else (4 if a.dtype == "float32" else 2)

        def factory():
            if spec.get("impl") != "native":
                raise RuntimeError(f"winner is the {spec.get('impl')} slot (no native plan)")
            opts = dict(spec.get("opts", {}))
            opts.pop("_env", None)
            opts["graph"] = False  # per-op events need the eager enqueue
            cls, o, _ = resolve(a.primitive, "native", opts)
            return cls(m=a.m, n=a.n, k=a.k, dtype=a.dtype, **o)

        from ddlb_amd.parallel.preflight import fused_rccl_cap

        res = diagnose.diagnose(comm, a.primitive, a.m, a.n, a.k, esz, factory,
                                budget_s=a.diag_budget_s,
                                caps=(0, fused_rccl_cap(max(comm.world_size, 2))))
        comm.destroy()
    except Exception as e:  # reported to the parent
        res["error"] = f"{type(e).__name__}: {str(e)[:300]}"
    with open(a.child_out, "w") as f:
        json.dump(res, f)
    return 0


def preflight_child(a) -> int:
    """One preflight family on this rank's GPU (progress file rewritten after every phase)."""
    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel import preflight

    try:
        comm = Communicator()
        comm.ensure_process_group(timeout_s=min(a.child_timeout, 60.0))
        if a.child_impl == "preflight_rccl":
            preflight.run_rccl_checks(comm, progress_path=a.child_out)
        else:
            preflight.run_ipc_checks(comm, progress_path=a.child_out)
        comm.destroy()
    except Exception as e:
        with open(a.child_out + ".err", "w") as f:
            f.write(f"{type(e).__name__}: {str(e)[:300]}")
    return 0


# ------------------------------------------------------------------------------- parent
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_count() -> int:
    """Visible GPUs, without initialising HIP in this (parent) process."""
    if os.environ.get("DDLB_DEVICE", "auto") == "cpu":
        return 0
    import torch

    return torch.cuda.device_count()


class Job:
    def __init__(self, a):
        self.a = a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.t_start = time.time()
        self.pg = None
        self.child_env = {}  # e.g. DDLB_PG_BACKEND=gloo when the RCCL control plane failed
        if self.world > 1:
            import datetime

            import torch.distributed as dist

            dist.init_process_group("gloo", init_method="env://", rank=self.rank,
                                    world_size=self.world,
                                    timeout=datetime.timedelta(seconds=3 * 3600))
            self.pg = dist
        self.tmp = os.environ.get("TMPDIR", "/tmp")
        self.counter = 0

    def log(self, msg: str) -> None:
        """Progress line on rank 0's stderr (the JSON result stays the only stdout line)."""
        if self.rank == 0:
            sys.stderr.write(f"[bench {time.time() - self.t_start:5.0f}s] {msg}\n")
            sys.stderr.flush()

    def left(self) -> float:
        """Seconds left before the job deadline (rank 0's clock; broadcast where it decides)."""
        return self.a.deadline_s - (time.time() - self.t_start)

    def bcast(self, obj):
        if self.pg is None:
            return obj
        box = [obj]
        self.pg.broadcast_object_list(box, src=0)
        return box[0]

    def gather(self, obj):
        if self.pg is None:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def _spawn(self, mode: str, opts: dict, timeout: float, extra=()):
        """Run one child per rank; returns (local result path, exit info). The timeout and the
        rendezvous port come from rank 0 so every rank kills its child at the same point."""
        self.counter += 1
        port, timeout = self.bcast((_free_port(), timeout) if self.rank == 0 else None)
        out = os.path.join(self.tmp, f"ddlb_bench_{os.getpid()}_{self.counter}.json")
        for p in (out, out + ".err"):
            if os.path.exists(p):
                os.remove(p)
        env = dict(os.environ)
        env.update(self.child_env)
        env["DDLB_CHILD_INIT_METHOD"] = f"tcp://127.0.0.1:{port}"
        opts = dict(opts)
        env.update(opts.pop("_env", {}))  # per-candidate runtime settings (e.g. RCCL channels)
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--child-out", out,
               "--child-impl", mode, "--child-opts", json.dumps(opts),
               "--primitive", self.a.primitive, "-m", str(self.a.m), "-n", str(self.a.n),
               "-k", str(self.a.k), "--dtype", self.a.dtype,
               "--child-timeout", str(max(timeout, 1.0)), *extra]
        # the child reports through --child-out; its stdout (RCCL's version banner, library
        # chatter) goes to stderr so the job's stdout holds the single JSON line only
        proc = subprocess.Popen(cmd, env=env, stdout=sys.stderr.fileno())
        status = "exit"
        try:
            proc.wait(timeout=max(timeout, 1.0))
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
            status = "timeout"
        return out, status, proc.returncode, timeout

    def measure(self, impl: str, opts: dict, steps: int, warmup: int, validate: bool,
                timeout: float, prewarm_ms: float = 0.0, harness_iters: int = 0) -> dict:
        """Run one measurement in a child per rank; every rank returns the same dict."""
        extra = ["--steps", str(steps), "--warmup", str(warmup), "--prewarm-ms",
                 str(prewarm_ms), "--harness-iters", str(harness_iters)]
        if validate:
            extra.append("--validate")
        out, status, rc, timeout = self._spawn(impl, opts, timeout, extra)
        if status == "timeout":
            local = {"ok": False, "error": f"timeout after {timeout:.0f}s"}
        elif os.path.exists(out):
            local = json.load(open(out))
        else:
            local = {"ok": False, "error": f"child exit {rc}"}
        if os.path.exists(out):
            os.remove(out)
        results = self.gather(local)
        if all(r.get("ok") for r in results):
            ms = max(r["ms"] for r in results)
            valid = all(r.get("valid") is not False for r in results)
            why = [r["validation"] for r in results if r.get("validation")]
            res = {"ok": True, "ms": ms, "valid": valid if validate else None,
                   "validation": why[0] if why else ""}
            errs = [r["max_err"] for r in results if "max_err" in r]
            if errs:
                res["max_err"] = max(errs)
                res["err_bound"] = min(r["err_bound"] for r in results if "err_bound" in r)
            cb = [r["copy_batch"] for r in results if "copy_batch" in r]
            if cb:
                res["copy_batch"] = cb[0]
            hm = [r["harness_mean_ms"] for r in results if "harness_mean_ms" in r]
            if hm:
                res["harness_mean_ms"] = max(hm)
            return res
        errs = [r.get("error") for r in results if not r.get("ok")]
        return {"ok": False, "error": errs[0] if errs else "unknown"}

    def diagnose(self, chosen, timeout: float) -> dict:
        """First-contact diagnostics (``diagnose_child``) in a child per rank: every rank's xGMI
        probe, rank 0's RCCL bus bandwidth and winner timeline (``diagnose.merge_ranks``)."""
        from ddlb_amd.parallel.diagnose import merge_ranks

        spec = {"impl": chosen[1], "opts": chosen[2]}
        out, status, rc, _ = self._spawn("diagnose", spec, timeout,
                                         ["--diag-budget-s", str(self.a.diag_budget_s)])
        local = None
        if status == "timeout":
            local = {"error": f"timeout after {timeout:.0f} s"}
        elif os.path.exists(out):
            local = json.load(open(out))
        else:
            local = {"error": f"child exit {rc}"}
        if os.path.exists(out):
            os.remove(out)
        return merge_ranks(self.gather(local))

    def preflight(self, timeout: float) -> dict:
        """Run the preflight families (RCCL, then IPC), each in its own child per rank."""
        from ddlb_amd.parallel import preflight as pf

        fake = os.environ.get("DDLB_PREFLIGHT_FAKE")
        if fake:  # tests: scripted results
            return json.loads(fake)
        if self.world == 1:
            return {"skipped": "world 1 (no cross-GPU data plane)"}
        if _gpu_count() == 0:
            return {"skipped": "no GPU visible"}
        merged = {}
        for mode, phases in (("preflight_rccl", pf.RCCL_PHASES), ("preflight_ipc", pf.IPC_PHASES)):
            t0 = time.time()
            env_saved = dict(self.child_env)
            self.child_env["DDLB_PG_BACKEND"] = "gloo"  # checks independent of torch's RCCL PG
            out, status, rc, _ = self._spawn(mode, {}, timeout)
            self.child_env = env_saved
            local = {}
            if os.path.exists(out):
                local = json.load(open(out))
            if os.path.exists(out + ".err"):
                local.setdefault("_error", open(out + ".err").read())
            for p in (out, out + ".err", out + ".tmp"):
                if os.path.exists(p):
                    os.remove(p)
            per_rank = self.gather(local)
            got = pf.merge(per_rank, phases)
            errs = [r.get("_error") for r in per_rank if r.get("_error")]
            if errs:
                for ph in phases:
                    if not got[ph].startswith("ok") and got[ph] == "failed: timeout":
                        got[ph] = f"failed: {errs[0][:160]}"
            merged.update(got)
            self.log(f"preflight {mode}: {json.dumps(got)} ({time.time() - t0:.1f} s)")
        return merged


def _blocked(opts_needs, pre: dict):
    """The first preflight check a candidate needs that did not pass (None = runnable)."""
    for ch in opts_needs:
        st = pre.get(ch)
        if st is not None and not str(st).startswith("ok"):
            return ch
    return None


def autotune(job, pool, a, world: int, tune: dict, pre: dict = None):
    """Time every candidate (validated) in its own children; returns (winner, fallbacks) or
    None when every candidate failed. ``tune`` collects per-candidate results for the report.
    Candidates needing a failed preflight check are skipped; a family whose candidates time out
    twice is skipped for the rest of the search (a hang costs the whole candidate timeout)."""
    from ddlb_amd.parallel.preflight import needs

    pre = pre or {}
    rounds = a.tune_rounds if a.tune_rounds > 0 else (2 if world == 1 else 1)
    tune_steps = a.tune_steps if a.tune_steps > 0 else (50 if world == 1 else 20)
    natives = [c for c in pool if c[1] == "native"]
    vendors = [c for c in pool if c[1] != "native"]
    order = natives * rounds + vendors  # the vendor slots once: they only feed vendor_ms
    best_ms = {}
    timeouts = {}
    t_tune = time.time()
    for label, impl, opts in order:
        req = needs(impl, opts, getattr(a, "primitive", "tp_columnwise"))
        why = _blocked(req, pre)
        if why is None:
            hung = [ch for ch in req if timeouts.get(ch, 0) >= 2]
            why = f"{hung[0]} candidates timed out twice" if hung else None
        if why is not None:
            tune.setdefault(label, f"skipped ({why})")
            continue
        # the search stops where the final run would no longer fit before the deadline (the
        # decision is rank 0's, broadcast, so every rank stops at the same candidate)
        native_ok = any(lb in best_ms for lb, _, _ in natives)
        spent = time.time() - t_tune
        room = job.left() - a.final_reserve_s
        over = (room < 10.0 or (native_ok and spent > a.tune_budget_s)
                or (best_ms and spent > a.tune_cap_s))
        if job.bcast(over if job.rank == 0 else None):
            tune.setdefault(label, "skipped (deadline / tuning budget)")
            continue
        t0 = time.time()
        # tuning runs validate too (first run and last timed step): a fast candidate that
        # computes the wrong numbers must never win the search
        r = job.measure(impl, opts, tune_steps, 3, a.validate,
                        min(a.candidate_timeout, max(room, 10.0)),
                        prewarm_ms=min(a.prewarm_ms, 100.0))
        if r["ok"] and r.get("valid") is False:
            r = {"ok": False, "error": f"invalid result: {r.get('validation', '')}"}
        if r["ok"]:
            best_ms[label] = min(r["ms"], best_ms.get(label, float("inf")))
            tune[label] = round(best_ms[label], 4)
        else:
            if r["error"].startswith("timeout") and req:
                # charged to the candidate's most specific mechanism (e.g. rccl_fused, ipc_agk):
                # two hangs of the RCCL-fed fused GEMM must not drop the plain RCCL pipelines
                timeouts[req[-1]] = timeouts.get(req[-1], 0) + 1
            if label not in best_ms:
                tune[label] = r["error"][:160]
        job.log(f"tune {label}: {round(r['ms'], 4) if r['ok'] else r['error'][:160]} "
                f"({time.time() - t0:.1f} s)")
    ranked = sorted(((best_ms[lb], (lb, i, o)) for lb, i, o in natives if lb in best_ms),
                    key=lambda x: x[0])
    vend = sorted(((best_ms[lb], (lb, i, o)) for lb, i, o in vendors if lb in best_ms),
                  key=lambda x: x[0])
    if not ranked:
        # every native path failed on this machine: report the vendor-library slot rather than
        # no number; the result line names the implementation and the library
        ranked = vend
        tune["native_failed"] = True
    if not ranked:
        return None
    chosen = ranked[0][1]
    fallbacks = [c for _, c in ranked[1:4]]
    # last resort: the vendor-library slot, so a job whose native paths all break in the
    # final run still reports a measured (and labelled) number
    if vend and vend[0][1] not in fallbacks and vend[0][1] is not chosen:
        fallbacks.append(vend[0][1])
    return chosen, fallbacks


def final_measure(job, chosen, fallbacks, a, tune: dict):
    """The timed measurement of the contract. Should the winner fail or not validate there (a
    flaky transport, a cross-rank ordering bug under back-to-back epochs), the next fastest
    candidates are tried while the deadline leaves room, so one bad path cannot sink the job.
    Returns (candidate, result); result is None if nothing ran, or has valid=False if nothing
    validated (then the first completed run is reported, with a nonzero exit code)."""
    invalid = None
    first = chosen
    for idx, cand in enumerate([chosen] + list(fallbacks)):
        room = job.left() - 5.0
        if job.bcast(room < 15.0 if job.rank == 0 else None):
            tune.setdefault("final_rejected", []).append(f"{cand[0]}: no time left (deadline)")
            break
        t0 = time.time()
        timeout = min(a.candidate_timeout + a.steps * 0.05 + a.harness_iters * 0.05, room)
        r = job.measure(cand[1], cand[2], a.steps, a.warmup, a.validate, timeout,
                        prewarm_ms=a.prewarm_ms, harness_iters=a.harness_iters)
        job.log(f"final {cand[0]}: {r.get('ms', r.get('error'))} valid={r.get('valid')} "
                f"({time.time() - t0:.1f} s)")
        if r["ok"] and r.get("valid") is not False:
            if cand is not first:
                tune["final_fallback_from"] = first[0]
            return cand, r
        if r["ok"] and invalid is None:
            invalid = (cand, r)
        tune.setdefault("final_rejected", []).append(
            f"{cand[0]}: {r.get('error') or 'invalid ' + r.get('validation', '')}"[:200])
    if invalid is not None:
        return invalid
    return chosen, None


def self_launch(gpus: int, argv) -> int:
    """``--gpus N`` without a launcher (no WORLD_SIZE): start ``torch.distributed.run`` with N
    ranks on this node as a CHILD process (this parent never touched the GPU, and never execs),
    relay the single JSON line of rank 0 and return the child's exit code. Rank discovery then
    follows the same env path as a torchrun launch (``/root/reference/ddlb/envs.py:50-67`` reads
    whatever launcher env is present)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(_free_port()), os.path.abspath(__file__), *argv]
    sys.stderr.write(f"[bench] --gpus {gpus} without a launcher: {' '.join(cmd[1:6])} ...\n")
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in proc.stdout:  # rank 0's JSON line to stdout, anything else to stderr
        out = sys.stdout if line.startswith("{") else sys.stderr
        out.write(line)
        out.flush()
    return proc.wait()


def json_stdout():
    """Reserve this process's stdout for the single JSON line: returns a file on a duplicate of
    fd 1 and points fd 1 at stderr, so whatever the libraries print to stdout (RCCL's version
    banner at every communicator init) cannot interleave with it."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("-m", type=int, default=65536)
    p.add_argument("-n", type=int, default=1024)
    p.add_argument("-k", type=int, default=1024)
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--primitive", default="tp_columnwise", choices=["tp_columnwise", "tp_rowwise"],
                   help="tp_columnwise = the flagship (AG+GEMM); tp_rowwise = GEMM+RS "
                        "(BASELINE config #3: -m 16384 -n 8192 -k 8192)")
    p.add_argument("--algorithm", default="auto",
                   help="auto | a candidate label (see CANDIDATES)")
    p.add_argument("--candidates", default="",
                   help="comma list of candidate labels to autotune over (default: all)")
    p.add_argument("--tune-steps", type=int, default=0,
                   help="timed steps per autotune measurement (0 = 50 at world 1, 20 otherwise)")
    p.add_argument("--tune-rounds", type=int, default=0,
                   help="passes over the native pool (0 = 2 at world 1, 1 otherwise)")
    p.add_argument("--candidate-timeout", type=float, default=45.0,
                   help="per-candidate child timeout (a healthy candidate takes ~3-15 s)")
    p.add_argument("--deadline-s", type=float, default=480.0,
                   help="wall-clock deadline of the WHOLE job (preflight, tuning, final run and "
                        "fallbacks): the driver allows 600 s")
    p.add_argument("--final-reserve-s", type=float, default=100.0,
                   help="time kept free of tuning for the final run and its fallbacks")
    p.add_argument("--preflight-timeout", type=float, default=40.0,
                   help="per-family timeout of the N>1 preflight children")
    p.add_argument("--tune-budget-s", type=float, default=300.0,
                   help="stop trying further candidates after this much autotuning wall time "
                        "(once a native candidate has succeeded)")
    p.add_argument("--tune-cap-s", type=float, default=360.0,
                   help="hard cap on autotuning wall time (once any candidate has succeeded)")
    p.add_argument("--no-validate", dest="validate", action="store_false", default=True)
    p.add_argument("--prewarm-ms", type=float, default=300.0,
                   help="untimed GPU pre-warm before the warmup steps (clock ramp)")
    p.add_argument("--preflight-only", action="store_true",
                   help="run the N>1 data-plane preflight, print its JSON line and exit")
    p.add_argument("--diagnose", choices=["auto", "on", "off"], default="auto",
                   help="first-contact diagnostics after the final run (xGMI probe, RCCL busbw "
                        "default vs capped, winner timeline) -> 'diag' in the JSON line; auto = "
                        "at world > 1")
    p.add_argument("--diag-budget-s", type=float, default=30.0,
                   help="wall-clock budget of the diagnostics' measurements")
    p.add_argument("--harness-iters", type=int, default=-1,
                   help="iterations of the reference-default timing (barrier before each, "
                        "MAX over ranks) after the timed window -> harness_mean_ms "
                        "(-1 = --steps, 0 = off)")
    # child-mode arguments (internal)
    p.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--child-out", help=argparse.SUPPRESS)
    p.add_argument("--child-impl", default="native", help=argparse.SUPPRESS)
    p.add_argument("--child-opts", default="{}", help=argparse.SUPPRESS)
    p.add_argument("--child-timeout", type=float, default=600.0, help=argparse.SUPPRESS)
    p.add_argument("--validate", dest="validate", action="store_true", help=argparse.SUPPRESS)
    a = p.parse_args(argv)
    if a.harness_iters < 0:
        a.harness_iters = a.steps
    if a.child:
        if a.child_impl.startswith("preflight_"):
            return preflight_child(a)
        if a.child_impl == "diagnose":
            return diagnose_child(a)
        return child_main(a)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(a.gpus, argv if argv is not None else sys.argv[1:])
    if a.gpus > 1 and world != a.gpus:
        sys.stderr.write(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks\n")
        return 2
    out = json_stdout()
    job = Job(a)
    # warm the page cache for the children: the first `import torch` on a fresh box takes 1-2
    # minutes, which would otherwise land inside the first candidate's timeout (importing torch
    # does not initialise the GPU in this parent)
    t0 = time.time()
    import torch  # noqa: F401
    job.log(f"import torch {time.time() - t0:.1f} s")
    tune = {}
    pool = candidate_pool(a.primitive, a.dtype, world)
    every = (candidate_pool(a.primitive, a.dtype, 1) +
             candidate_pool(a.primitive, a.dtype, 2, extra=True))
    if a.candidates:
        want = [c.strip() for c in a.candidates.split(",") if c.strip()]
        unknown = [w for w in want if w not in [c[0] for c in every]]
        if unknown:
            raise SystemExit(f"unknown candidates {unknown}")
        pool = [c for c in every if c[0] in want]
    pre = job.preflight(min(a.preflight_timeout, max(job.left() / 4, 10.0)))
    if a.preflight_only:
        if job.rank == 0:
            print(json.dumps({"preflight": pre, "n_gpus": world}), file=out, flush=True)
        if job.pg is not None:
            job.pg.destroy_process_group()
        return 0 if all(str(v).startswith("ok") for v in pre.values()) else 1
    if not str(pre.get("torch_nccl", "ok")).startswith("ok"):
        # torch's RCCL group is broken on this node: the children coordinate over gloo (the
        # control plane: barriers, the MAX over ranks), our native data plane is unaffected
        job.child_env["DDLB_PG_BACKEND"] = "gloo"
    fallbacks = []
    if a.algorithm != "auto":
        match = [c for c in every if c[0] == a.algorithm]
        if not match:
            raise SystemExit(f"unknown --algorithm {a.algorithm}; choose from "
                             f"{[c[0] for c in every]}")
        chosen = match[0]
    else:
        picked = autotune(job, pool, a, world, tune, pre)
        if picked is None:
            sys.stderr.write(f"every candidate failed: {json.dumps(tune)}\n")
            return 1
        chosen, fallbacks = picked
    chosen, final = final_measure(job, chosen, fallbacks, a, tune)
    if final is None:
        sys.stderr.write(f"final measurement failed (autotune: {json.dumps(tune)})\n")
        return 1
    diag = None
    if a.diagnose == "on" or (a.diagnose == "auto" and world > 1):
        # bounded: the measurements' own budget plus child start-up, and never past the deadline
        room = job.left() - 5.0
        if job.bcast(room < a.diag_budget_s + 15.0 if job.rank == 0 else None):
            diag = {"skipped": f"deadline ({room:.0f} s left)"}
        else:
            t0 = time.time()
            diag = job.diagnose(chosen, min(a.diag_budget_s + 45.0, room))
            diag["job_s"] = round(time.time() - t0, 1)
            job.log(f"diagnostics: {json.dumps(diag)[:600]} ({diag['job_s']} s)")
    ms = final["ms"]
    flop = 2.0 * a.m * a.n * a.k
    harness_tflops = flop / (ms * 1e-3) / 1e12  # the reference's formula (ddlb/benchmark.py:211)
    col = a.primitive == "tp_columnwise"
    # whole-job aggregate: tp_columnwise = every rank computes the full [m,k]x[k,n] on its own
    # N-slice (weak scaling, N x the harness number); tp_rowwise = the ranks share one
    # [m,k]x[k,n] split along K (strong scaling, the harness number IS the aggregate)
    value = harness_tflops * world if col else harness_tflops
    vendor = {lbl: tune[lbl] for lbl, impl, _ in pool
              if impl != "native" and isinstance(tune.get(lbl), float)}
    if job.rank == 0:
        dt = {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32",
              "float8_e4m3fn": "fp8_e4m3"}.get(a.dtype, a.dtype)
        native = chosen[1] == "native"
        line = {
            "metric": (f"tp_columnwise AG+GEMM effective TFLOP/s (whole job, m={a.m} {dt})" if col
                       else f"tp_rowwise GEMM+RS effective TFLOP/s (whole job, m={a.m} {dt})"),
            "value": round(value, 6), "unit": "TFLOP/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 5),
            "higher_is_better": True, "scaling": "weak" if col else "strong",
            "vs_baseline": None, "dtype": dt, "data": "synthetic",
            "config": {"model": (f"tp_columnwise AG+GEMM m={a.m} n={a.n} k={a.k}" if col
                                 else f"tp_rowwise GEMM+RS m={a.m} n={a.n} k={a.k}"),
                       "global_batch": 1, "seq_len": a.m, "parallelism": f"tp{world}-sp",
                       "implementation": chosen[1], "algorithm": chosen[0]},
            "per_gpu_tflops": round(harness_tflops if col else harness_tflops / world, 6),
            "harness_tflops": round(harness_tflops, 6), "valid": final.get("valid"),
            "gemm": "ddlb_amd MFMA" if native else "hipblaslt (vendor slot: every native failed)",
            "timing": TIMING,
            "harness_mean_ms": (round(final["harness_mean_ms"], 5)
                                if "harness_mean_ms" in final else None),
            "harness_timing": "reference default: cpu_clock, barrier before every iteration, "
                              "MAX over ranks per iteration (ddlb/benchmark.py:161-172)",
            "max_err": final.get("max_err"), "err_bound": final.get("err_bound"),
            "copy_batch": final.get("copy_batch"),
            "vendor_ms": vendor,
            "preflight": pre,
            "prewarm_ms": a.prewarm_ms,
            "deadline_s": a.deadline_s, "job_wall_s": round(time.time() - job.t_start, 1),
            "autotune_ms": tune,
        }
        if diag is not None:
            line["diag"] = diag
        print(json.dumps(line), file=out, flush=True)
    if job.pg is not None:
        job.pg.destroy_process_group()
    return 0 if final.get("valid") is not False else 1


if __name__ == "__main__":
    sys.exit(main())
