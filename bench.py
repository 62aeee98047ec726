#!/usr/bin/env python3
"""Flagship benchmark: tp_columnwise AG+GEMM, m=65536 (sequence), n=1024, k=1024, bf16.

BASELINE.json metric: "ms/iter + effective TFLOP/s, tp_columnwise AG+GEMM m=65536 bf16 at
1/2/4/8 GPUs". n=k=1024 is the reference README's m=65536 example (``README.md:37-39``).

Contract (driver):  python bench.py --gpus N --steps K --warmup W
  * N>1 is launched by torch.distributed.run, one rank per GPU (RANK/LOCAL_RANK/WORLD_SIZE env);
  * W untimed warmups, then EXACTLY K timed steps bracketed by barrier + device sync on both
    sides; ms_per_step is the MAX over ranks;
  * rank 0 prints ONE JSON line. ``value`` = whole-job effective TFLOP/s = N * 2*m*n*k / t
    (every rank computes the full [m,k]x[k,n] on its own N-slice of the weight: weak scaling in
    N); ``per_gpu_tflops`` is the reference harness's per-GPU number (``ddlb/benchmark.py:211``).

Other BASELINE configs through the same machinery: ``--primitive tp_rowwise -m 16384 -n 8192
-k 8192`` (config #3, GEMM + reduce-scatter; strong scaling: the harness number is the whole-job
aggregate) and ``--dtype float8_e4m3fn`` (config #5; adds the block-scaled MX-fp8 candidates).

Process model (robust by construction): the launched processes never touch the GPU. They form
a gloo group and run every measurement in a child process per rank (fresh HIP context, its own
rendezvous port, a hard timeout). An autotuner first times each candidate algorithm in its own
children (MAX over ranks), then the winner runs the timed measurement (falling back to the next
fastest if it fails there); a candidate that fails or hangs is killed and skipped on every rank,
so one bad path cannot hang the job. Every rank issues the same number of run() calls (the
pre-warm count is MAX-reduced), as each call holds collectives / epoch-matched signals.
Candidate timings are reported in the JSON (``autotune_ms``), progress on stderr. Synthetic
U[-1,1) inputs of the named shape (no datasets exist offline); the result is validated against
an fp32 reference.
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

# (label, impl, options). "/blas" = the plan's plain GEMM ops on hipBLASLt (gemm_mode=blas),
# everything else identical.
def _blas(opts):
    return dict(opts, gemm_mode="blas")


_COLL4 = dict(algorithm="coll_pipeline", backend="rccl", s=4)
_DEF = dict(algorithm="default", backend="rccl")
_P2P = dict(algorithm="p2p_pipeline", backend="ipc", multicast_protocol="memcpy")
_COLL_IPC = dict(algorithm="coll_pipeline", backend="ipc", multicast_protocol="memcpy", s=4)
_DEF_K = dict(algorithm="default", backend="ipc", multicast_protocol="kernel", copy_blocks=128)
# Pipeline stages use grouped-row GEMMs, which stay on the MFMA kernels (hipBLASLt only takes
# plain GEMMs), so coll_pipeline has no "/blas" twin.
# Flag-gated ("fused") GEMMs: ONE GEMM launch whose tiles spin until their rows have landed.
# With ranks sharing one GPU (the only multi-rank rehearsal available here) the spinning tiles of
# one rank hold the CUs the other needs and ran 30-100x slower (profiles/r01/s2/); on a real node
# each rank owns its GPU and the copy engines fill the flags without any CU, so the block-major
# fused coll_pipeline (no per-stage GEMM tails, one launch) stays in the pool. The whole-shard
# p2p form stays a CLI option (a tile waits for its entire 1/d shard).


def _graph(opts):
    return dict(opts, graph=True)


# Ordered by expected strength at d = 8 (the tuning budget may cut the tail of the list).
# "/graph": the whole plan is captured once and replayed with one hipGraphLaunch per run; the
# IPC pipelines issue one HIP call per copy / event / signal (~2 us of host time each, ~200 calls
# per run at d = 8, s = 8: host-bound without the graph, profiles/r02/r2_13_*).
# In-kernel all-gather ("agk"): ONE launch per run; its first copy_blocks workgroups pull the
# peers' row blocks over xGMI and flag them, the rest run the persistent GEMM gated on the flags
# (no copy streams, no host op per block, one kernel to capture).
_AGK = dict(algorithm="coll_pipeline", backend="ipc", multicast_protocol="kernel", fused=True,
            s=8, copy_blocks=32)
CANDIDATES = [
    ("coll_pipeline/rccl/s4", "native", _COLL4),
    ("coll_pipeline/ipc/agk32/s8/graph", "native", _graph(_AGK)),
    ("coll_pipeline/ipc/agk64/s8/graph", "native", _graph(dict(_AGK, copy_blocks=64))),
    ("coll_pipeline/ipc/memcpy/s8/graph", "native", _graph(dict(_COLL_IPC, s=8))),
    ("coll_pipeline/ipc/kernel/s8/graph", "native", _graph(dict(
        _COLL_IPC, s=8, multicast_protocol="kernel", copy_blocks=128, tile="128x128"))),
    ("coll_pipeline/ipc/memcpy/s8/fused/graph", "native", _graph(dict(_COLL_IPC, s=8,
                                                                      fused=True))),
    ("direct/ipc", "native", dict(algorithm="direct", backend="ipc")),
    ("coll_pipeline/ipc/memcpy/s4/fused/graph", "native", _graph(dict(_COLL_IPC, fused=True))),
    ("coll_pipeline/ipc/memcpy/s4/graph", "native", _graph(_COLL_IPC)),
    # each peer's chunks split over 2 copy streams (2 copy engines per link): a hedge for links
    # faster than one engine, which is what bounds the few-GPU runs (one link per peer); not
    # graph-captured (hipGraph replay of split copies segfaulted, profiles/r02/r2_22_*)
    ("coll_pipeline/ipc/memcpy/s8/cs2", "native", dict(_COLL_IPC, s=8, copy_streams=2)),
    # Stage GEMMs next to CU-resident comm kernels (our copy kernel): 128x128 tiles (4x as many,
    # dispatched dynamically) let the CUs busy with copies simply take fewer of them
    ("coll_pipeline/ipc/kernel/s4", "native", dict(_COLL_IPC, multicast_protocol="kernel",
                                                   copy_blocks=128, tile="128x128")),
    ("default/rccl", "native", _DEF),
    ("default/rccl/blas", "native", _blas(_DEF)),
    ("p2p_pipeline/ipc/memcpy/graph", "native", _graph(_P2P)),
    ("p2p_pipeline/ipc/memcpy/cs2", "native", dict(_P2P, copy_streams=2)),
    # HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default); the
    # memcpy protocol uses one copy stream per peer (9 streams at d=8): a variant where no two of
    # its streams share a queue (one process per GPU here, so 12 queues on the device)
    ("coll_pipeline/ipc/memcpy/s8/q12", "native", dict(_COLL_IPC, s=8,
                                                        _env={"GPU_MAX_HW_QUEUES": "12"})),
    ("coll_pipeline/ipc/memcpy/s8", "native", dict(_COLL_IPC, s=8)),
    ("coll_pipeline/ipc/agk32/s4/graph", "native", _graph(dict(_AGK, s=4))),
    ("coll_pipeline/ipc/agk32/s8", "native", _AGK),
    ("default/ipc/kernel", "native", _DEF_K),
    # the same reasoning for RCCL's CU-resident kernels, and RCCL held to 16 channels (16 CUs)
    ("coll_pipeline/rccl/s4/128", "native", dict(_COLL4, tile="128x128")),
    ("coll_pipeline/rccl/s8", "native", dict(_COLL4, s=8)),
    ("coll_pipeline/rccl/s8/128", "native", dict(_COLL4, s=8, tile="128x128")),
    ("coll_pipeline/rccl/s4/128/c16", "native", dict(_COLL4, tile="128x128",
                                                      _env={"NCCL_MAX_NCHANNELS": "16"})),
    ("coll_pipeline/ipc/kernel/s8", "native", dict(_COLL_IPC, s=8, multicast_protocol="kernel",
                                                   copy_blocks=128, tile="128x128")),
    ("coll_pipeline/ipc/memcpy/s4", "native", _COLL_IPC),
    ("p2p_pipeline/ipc/memcpy", "native", _P2P),
    ("p2p_pipeline/ipc/push", "native", dict(_P2P, direction="push")),
    ("default/ipc/push", "native", dict(_P2P, algorithm="default", direction="push")),
    ("coll_pipeline/ipc/push/s4", "native", dict(_COLL_IPC, direction="push")),
    ("default/ipc/kernel/push", "native", dict(_DEF_K, direction="push")),
    ("p2p_pipeline/rccl", "native", dict(algorithm="p2p_pipeline", backend="rccl")),
    # kernel-side flags (one spin / store kernel for all flags of an op instead of one rocclr
    # stream-memop kernel per flag)
    ("default/ipc/kernel/ksig", "native", dict(_DEF_K, signal="kernel")),
    ("pytorch(rccl+hipblaslt)", "pytorch", dict(backend="nccl", empty_cache=False)),
]
# world 1: the all-gather is the identity; the plan is one GEMM on either kernel family
WORLD1 = [
    ("gemm (world=1)/hip", "native", _DEF),
    ("gemm (world=1)/blas", "native", _blas(_DEF)),
]
# tp_rowwise (GEMM + sequence-parallel reduce-scatter; BASELINE config #3)
_RK = dict(backend="ipc", multicast_protocol="kernel", copy_blocks=128)
ROW_CANDIDATES = [
    ("row/default/rccl", "native", dict(algorithm="default", backend="rccl")),
    ("row/default/rccl/blas", "native", _blas(dict(algorithm="default", backend="rccl"))),
    ("row/coll_pipeline/rccl/s4", "native", dict(algorithm="coll_pipeline", backend="rccl", s=4)),
    ("row/coll_pipeline/rccl/s4/128", "native", dict(algorithm="coll_pipeline", backend="rccl",
                                                     s=4, tile="128x128")),
    ("row/p2p_pipeline/rccl", "native", dict(algorithm="p2p_pipeline", backend="rccl")),
    ("row/default/ipc/kernel", "native", dict(_RK, algorithm="default")),
    ("row/default/ipc/kernel/blas", "native", _blas(dict(_RK, algorithm="default"))),
    ("row/coll_pipeline/ipc/kernel/s4", "native", dict(_RK, algorithm="coll_pipeline", s=4)),
    # direct store: ONE GEMM whose epilogue writes every peer's partial into its receive slot
    # over xGMI (shard-interleaved tiles: all links at once), then one local d-way reduce
    ("row/p2p_pipeline/ipc/direct/graph", "native", _graph(dict(algorithm="p2p_pipeline",
                                                                backend="ipc", fused=True))),
    ("row/p2p_pipeline/ipc/direct", "native", dict(algorithm="p2p_pipeline", backend="ipc",
                                                   fused=True)),
    ("row/p2p_pipeline/ipc/memcpy", "native", dict(algorithm="p2p_pipeline", backend="ipc")),
    ("row/coll_pipeline/ipc/kernel/s4/graph", "native", _graph(dict(_RK, algorithm="coll_pipeline",
                                                                    s=4))),
    ("row/p2p_pipeline/ipc/memcpy/graph", "native", _graph(dict(algorithm="p2p_pipeline",
                                                                 backend="ipc"))),
    ("row/pytorch(rccl+hipblaslt)", "pytorch", dict(backend="nccl", empty_cache=False)),
]
ROW_WORLD1 = [
    ("row/gemm (world=1)/hip", "native", dict(algorithm="default", backend="rccl")),
    ("row/gemm (world=1)/blas", "native", _blas(dict(algorithm="default", backend="rccl"))),
]


def candidate_pool(primitive: str, dtype: str, world: int):
    """(label, impl, options) list for one primitive / dtype / world size. fp8 inputs add the
    block-scaled MX-fp8 MFMA (2x the bf16 rate) and drop hipBLASLt (no fp8 in the plain path)."""
    if primitive == "tp_rowwise":
        pool = ROW_WORLD1 if world == 1 else ROW_CANDIDATES
    else:
        pool = WORLD1 if world == 1 else CANDIDATES
    if dtype == "float8_e4m3fn":
        pool = [c for c in pool if c[2].get("gemm_mode") != "blas"]
        pool = pool + [(lbl + "/mx", impl, dict(opts, gemm_mode="mx")) for lbl, impl, opts in pool
                       if impl == "native"]
    return pool


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
    """Validate one output; a mismatch is recorded in ``res`` (not raised)."""
    try:
        impl.validate(out)
        return True
    except AssertionError as e:
        res["validation"] = str(e).splitlines()[0][:200]
        return False


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
        res.update(ok=True, ms=float(t.item()), valid=valid)
        impl.close()
        comm.destroy()
    except Exception as e:  # reported to the parent, never raised
        res["error"] = f"{type(e).__name__}: {str(e)[:300]}"
    with open(a.child_out, "w") as f:
        json.dump(res, f)
    return 0


# ------------------------------------------------------------------------------- parent
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Job:
    def __init__(self, a):
        self.a = a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.pg = None
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
            sys.stderr.write(f"[bench] {msg}\n")
            sys.stderr.flush()

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

    def measure(self, impl: str, opts: dict, steps: int, warmup: int, validate: bool,
                timeout: float, prewarm_ms: float = 0.0) -> dict:
        """Run one measurement in a child per rank; every rank returns the same dict."""
        self.counter += 1
        port = self.bcast(_free_port() if self.rank == 0 else None)
        out = os.path.join(self.tmp, f"ddlb_bench_{os.getpid()}_{self.counter}.json")
        env = dict(os.environ)
        env["DDLB_CHILD_INIT_METHOD"] = f"tcp://127.0.0.1:{port}"
        opts = dict(opts)
        env.update(opts.pop("_env", {}))  # per-candidate runtime settings (e.g. RCCL channels)
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--child-out", out,
               "--child-impl", impl, "--child-opts", json.dumps(opts), "--steps", str(steps),
               "--warmup", str(warmup), "--primitive", self.a.primitive,
               "-m", str(self.a.m), "-n", str(self.a.n), "-k",
               str(self.a.k), "--dtype", self.a.dtype, "--child-timeout", str(timeout),
               "--prewarm-ms", str(prewarm_ms)]
        if validate:
            cmd.append("--validate")
        proc = subprocess.Popen(cmd, env=env)
        try:
            proc.wait(timeout=timeout)
            local = json.load(open(out)) if os.path.exists(out) else {
                "ok": False, "error": f"child exit {proc.returncode}"}
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
            local = {"ok": False, "error": f"timeout after {timeout:.0f}s"}
        finally:
            if os.path.exists(out):
                os.remove(out)
        results = self.gather(local)
        if all(r.get("ok") for r in results):
            ms = max(r["ms"] for r in results)
            valid = all(r.get("valid") is not False for r in results)
            why = [r["validation"] for r in results if r.get("validation")]
            return {"ok": True, "ms": ms, "valid": valid if validate else None,
                    "validation": why[0] if why else ""}
        errs = [r.get("error") for r in results if not r.get("ok")]
        return {"ok": False, "error": errs[0] if errs else "unknown"}


def autotune(job, pool, a, world: int, tune: dict):
    """Time every candidate (validated) in its own children; returns (winner, fallbacks) or
    None when every candidate failed. ``tune`` collects per-candidate results for the report."""
    t_tune = time.time()
    rounds = a.tune_rounds if a.tune_rounds > 0 else (2 if world == 1 else 1)
    tune_steps = a.tune_steps if a.tune_steps > 0 else (50 if world == 1 else 20)
    best_ms = {}
    # several rounds over the pool in the same order, best time per candidate: a candidate
    # measured first after an idle gap otherwise pays the clock ramp the others do not
    for label, impl, opts in pool * rounds:
        # wall-clock cap on the search (the decision is broadcast from rank 0, so every
        # rank stops at the same candidate): the best candidate so far runs the final
        native_ok = any(lb in best_ms for lb, i, _ in pool if i == "native")
        spent = time.time() - t_tune
        over = (native_ok and spent > a.tune_budget_s) or (best_ms and spent > a.tune_cap_s)
        if job.bcast(over if job.rank == 0 else None):
            tune.setdefault(label, "skipped (tuning budget)")
            continue
        t0 = time.time()
        # tuning runs validate too (first run and last timed step): a fast candidate that
        # computes the wrong numbers must never win the search
        r = job.measure(impl, opts, tune_steps, 3, a.validate, a.candidate_timeout,
                        prewarm_ms=min(a.prewarm_ms, 100.0))
        if r["ok"] and r.get("valid") is False:
            r = {"ok": False, "error": f"invalid result: {r.get('validation', '')}"}
        if r["ok"]:
            best_ms[label] = min(r["ms"], best_ms.get(label, float("inf")))
            tune[label] = round(best_ms[label], 4)
        elif label not in best_ms:
            tune[label] = r["error"][:160]
        job.log(f"tune {label}: {round(r['ms'], 4) if r['ok'] else r['error'][:160]} "
                f"({time.time() - t0:.1f} s)")
    ranked = [(best_ms[label], (label, impl, opts)) for label, impl, opts in pool
              if impl == "native" and label in best_ms]
    if not ranked:
        # every native path failed on this machine: report the vendor-library slot (our
        # pytorch implementation, RCCL + hipBLASLt) rather than no number; the result line
        # names the implementation
        ranked = [(best_ms[label], (label, impl, opts)) for label, impl, opts in pool
                  if label in best_ms]
        tune["native_failed"] = True
    if not ranked:
        return None
    ranked.sort(key=lambda x: x[0])
    chosen = ranked[0][1]
    fallbacks = [c for _, c in ranked[1:4]]
    # last resort: the vendor-library slot, so a job whose native paths all break in the
    # final run still reports a measured (and labelled) number
    vendor = sorted(((best_ms[lbl], (lbl, i, o)) for lbl, i, o in pool
                     if i != "native" and lbl in best_ms), key=lambda x: x[0])
    if vendor and vendor[0][1] not in fallbacks and vendor[0][1] is not chosen:
        fallbacks.append(vendor[0][1])
    return chosen, fallbacks


def final_measure(job, chosen, fallbacks, a, tune: dict):
    """The timed measurement of the contract. Should the winner fail or not validate there (a
    flaky transport, a cross-rank ordering bug under back-to-back epochs), the next fastest
    candidates are tried before giving up, so one bad path cannot sink the job. Returns
    (candidate, result); result is None if nothing ran, or has valid=False if nothing
    validated (then the first completed run is reported, with a nonzero exit code)."""
    final, invalid = None, None
    first = chosen
    for cand in [chosen] + list(fallbacks):
        t0 = time.time()
        r = job.measure(cand[1], cand[2], a.steps, a.warmup, a.validate,
                        a.candidate_timeout + a.steps * 0.05, prewarm_ms=a.prewarm_ms)
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
    return chosen, final


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
                   help="passes over the candidate pool (0 = 2 at world 1, 1 otherwise)")
    p.add_argument("--candidate-timeout", type=float, default=60.0,
                   help="per-candidate child timeout (a healthy candidate takes ~3-15 s)")
    p.add_argument("--tune-budget-s", type=float, default=300.0,
                   help="stop trying further candidates after this much autotuning wall time "
                        "(once a native candidate has succeeded); sized so the whole job, "
                        "final run and fallbacks included, stays well inside 10 minutes")
    p.add_argument("--tune-cap-s", type=float, default=420.0,
                   help="hard cap on autotuning wall time (once any candidate has succeeded)")
    p.add_argument("--no-validate", dest="validate", action="store_false", default=True)
    p.add_argument("--prewarm-ms", type=float, default=300.0,
                   help="untimed GPU pre-warm before the warmup steps (clock ramp)")
    # child-mode arguments (internal)
    p.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--child-out", help=argparse.SUPPRESS)
    p.add_argument("--child-impl", default="native", help=argparse.SUPPRESS)
    p.add_argument("--child-opts", default="{}", help=argparse.SUPPRESS)
    p.add_argument("--child-timeout", type=float, default=600.0, help=argparse.SUPPRESS)
    p.add_argument("--validate", dest="validate", action="store_true", help=argparse.SUPPRESS)
    a = p.parse_args(argv)
    if a.child:
        return child_main(a)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and world == 1:
        sys.stderr.write("bench.py: --gpus > 1 must be launched with torch.distributed.run\n")
        return 2
    job = Job(a)
    tune = {}
    pool = candidate_pool(a.primitive, a.dtype, world)
    every = candidate_pool(a.primitive, a.dtype, 1) + candidate_pool(a.primitive, a.dtype, 2)
    if a.candidates:
        want = [c.strip() for c in a.candidates.split(",") if c.strip()]
        unknown = [w for w in want if w not in [c[0] for c in every]]
        if unknown:
            raise SystemExit(f"unknown candidates {unknown}")
        pool = [c for c in every if c[0] in want]
    fallbacks = []
    if a.algorithm != "auto":
        match = [c for c in every if c[0] == a.algorithm]
        if not match:
            raise SystemExit(f"unknown --algorithm {a.algorithm}; choose from "
                             f"{[c[0] for c in every]}")
        chosen = match[0]
    else:
        picked = autotune(job, pool, a, world, tune)
        if picked is None:
            sys.stderr.write(f"every candidate failed: {json.dumps(tune)}\n")
            return 1
        chosen, fallbacks = picked
    chosen, final = final_measure(job, chosen, fallbacks, a, tune)
    if final is None:
        sys.stderr.write(f"final measurement failed (autotune: {json.dumps(tune)})\n")
        return 1
    ms = final["ms"]
    flop = 2.0 * a.m * a.n * a.k
    harness_tflops = flop / (ms * 1e-3) / 1e12  # the reference's formula (ddlb/benchmark.py:211)
    col = a.primitive == "tp_columnwise"
    # whole-job aggregate: tp_columnwise = every rank computes the full [m,k]x[k,n] on its own
    # N-slice (weak scaling, N x the harness number); tp_rowwise = the ranks share one
    # [m,k]x[k,n] split along K (strong scaling, the harness number IS the aggregate)
    value = harness_tflops * world if col else harness_tflops
    if job.rank == 0:
        dt = {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32",
              "float8_e4m3fn": "fp8_e4m3"}.get(a.dtype, a.dtype)
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
            "gemm": ("hipblaslt" if chosen[1] == "pytorch" or chosen[2].get("gemm_mode") == "blas"
                     else "ddlb_amd MFMA"),
            "prewarm_ms": a.prewarm_ms,
            "autotune_ms": tune,
        }
        print(json.dumps(line), flush=True)
    if job.pg is not None:
        job.pg.destroy_process_group()
    return 0 if final.get("valid") is not False else 1


if __name__ == "__main__":
    sys.exit(main())
