"""Benchmark runner: one isolated child process per (shape, implementation config).

Parity: ``ddlb/benchmark.py`` — ``_benchmark_worker_entry`` (:19-256) and
``PrimitiveBenchmarkRunner`` (:264-389). Reproduced exactly:

* warmups, a profiler window of 5 ``run()`` calls, warmups again, then the timed loop
  (``2*num_warmups + 5 + num_iterations`` calls in total);
* the four timing modes: ``cpu_clock``/``cuda_event`` x barrier/no-barrier (:124-188);
* the per-iteration times vector is MAX-all-reduced across ranks (:190-204);
* mean / population-std / min / max and TFLOPS ``2mnk/(t_ms*1e9)`` (:206-214);
* validation of the last result, recorded as ``valid`` (:239-245);
* rank 0 prints every row and appends it to the CSV immediately (:372-384).

Closed gaps: the parent waits with a timeout and records a
``valid=False, error=...`` row when a child dies or hangs; each child gets its own
rendezvous port; a construction or run error becomes an error row instead of a hang;
``resume=True`` skips rows already present in the CSV.
"""

from __future__ import annotations

import csv
import json
import os
import queue as _queue
import socket
import subprocess
import sys
import time
import traceback
from typing import Any, Dict, List, Optional

from ddlb_amd.envs import get_master_addr, get_master_port, get_rank, get_world_size
from ddlb_amd.utils.stats import CSV_COLUMNS, EXTRA_COLUMNS, derived_metrics, impl_label, \
    option_string, order_row, summarize


def _spec_key(impl_opts: Dict[str, Any]) -> str:
    return json.dumps(impl_opts, sort_keys=True, default=str)


def _time_loop(impl, comm, backend: str, barrier: bool, iters: int):
    """Return (times_ms, last_result). Mirrors ``ddlb/benchmark.py:124-188``."""
    import torch
    import torch.distributed as dist

    times: List[float] = []
    last = None
    if backend == "cuda_event" and not comm.is_gpu:
        backend = "cpu_clock"
    if backend == "cuda_event":
        if barrier:
            starts = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
            ends = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
            dummy = torch.zeros(1, dtype=torch.int32, device=comm.device)
            for i in range(iters):
                if dist.is_initialized():
                    dist.all_reduce(dummy)
                    torch.cuda.synchronize()
                starts[i].record()
                last = impl.run()
                ends[i].record()
            torch.cuda.synchronize()
            times = [starts[i].elapsed_time(ends[i]) for i in range(iters)]
        else:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(iters):
                last = impl.run()
            e.record()
            torch.cuda.synchronize()
            times = [s.elapsed_time(e) / iters] * iters
    elif backend == "cpu_clock":
        if barrier:
            for _ in range(iters):
                comm.barrier()
                t0 = time.perf_counter()
                last = impl.run()
                comm.synchronize()
                times.append((time.perf_counter() - t0) * 1e3)
        else:
            comm.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                last = impl.run()
            comm.synchronize()
            times = [(time.perf_counter() - t0) * 1e3 / iters] * iters
    else:
        raise ValueError(f"Unknown time_measurement_backend: {backend}")
    return times, last


def run_single(primitive: str, impl_id: str, m: int, n: int, k: int, dtype: str,
               num_warmups: int, num_iterations: int, impl_opts: Dict[str, Any],
               validate: bool, time_measurement_backend: str = "cpu_clock",
               barrier_at_each_iteration: bool = True, profile_iterations: int = 5,
               validate_every_iteration: bool = False) -> Dict[str, Any]:
    """Construct, warm up, profile-window, time, MAX-reduce, validate. Returns the row.

    Runs in the calling process (the runner calls it inside the spawned child)."""
    import torch

    from ddlb_amd.cli.config import base_impl_name
    from ddlb_amd.communicator import Communicator
    from ddlb_amd.primitives.registry import resolve
    from ddlb_amd.utils import profiling

    base = impl_opts.get("implementation") or base_impl_name(impl_id)
    cls, options, note = resolve(primitive, base, impl_opts)
    if note and get_rank() == 0:
        print(f"[ddlb_amd] {note}")
    comm = Communicator()
    comm.ensure_process_group()
    default_keys = list(getattr(cls, "DEFAULT_OPTIONS", {}).keys())
    row: Dict[str, Any] = {
        "implementation": base, "m": m, "n": n, "k": k, "dtype": dtype,
        "world_size": get_world_size(), "hostname": socket.gethostname(),
        "time_measurement_backend": time_measurement_backend,
        "barrier_at_each_iteration": barrier_at_each_iteration, "option": "",
    }
    impl = None
    try:
        impl = cls(m=m, n=n, k=k, dtype=dtype, **options)
        opts_used = impl.options.as_dict()
        row["implementation"] = impl_label(base, opts_used, default_keys)
        row["option"] = option_string(opts_used, default_keys)
        for _ in range(num_warmups):
            impl.run()
        comm.synchronize()
        profiling.profiler_resume()
        for _ in range(profile_iterations):
            with profiling.roctx_range(row["implementation"]):
                impl.run()
        comm.synchronize()
        profiling.profiler_pause()
        for _ in range(num_warmups):
            impl.run()
        if validate_every_iteration:
            def _checked():
                r = impl.run()
                impl.validate(r)
                return r
            checked = type("Checked", (), {"run": staticmethod(_checked)})()
            times, last = _time_loop(checked, comm, time_measurement_backend,
                                     barrier_at_each_iteration, num_iterations)
        else:
            times, last = _time_loop(impl, comm, time_measurement_backend,
                                     barrier_at_each_iteration, num_iterations)
        t = torch.tensor(times, dtype=torch.float64, device=comm.device)
        comm.all_reduce_max(t)
        # a device-side bounded wait that gave up during warmup / timing means some step ran on
        # stale data: an error row even when validation is off
        impl.check_health()
        times = t.cpu().tolist()
        row.update(summarize(times, m, n, k))
        row.update(derived_metrics(primitive, base, str(opts_used.get("size", "")), m, n, k, dtype,
                                   get_world_size(), row["mean_time (ms)"]))
        if validate and last is not None:
            try:
                impl.validate(last)
                row["valid"] = True
            except Exception as e:  # numerics failure is recorded, not fatal
                row["valid"] = False
                row["error"] = f"validation: {str(e).splitlines()[0][:300]}"
                if get_rank() == 0:
                    print(f"Warning: Validation failed for {impl_id} with error: {e}")
    except Exception as e:
        row.update(summarize([], m, n, k))
        row["valid"] = False
        row["error"] = f"{type(e).__name__}: {str(e).splitlines()[0][:300] if str(e) else ''}"
        if os.environ.get("DDLB_TRACEBACK", "1") == "1":
            traceback.print_exc()
    finally:
        if impl is not None:
            try:
                impl.close()
            except Exception:
                pass
            del impl
        if comm.is_gpu:
            try:
                torch.cuda.empty_cache()
            except Exception:
                pass
    row["gpu_arch"] = _gpu_arch(comm)
    row.setdefault("error", "")
    return row


def _gpu_arch(comm) -> str:
    if not comm.is_gpu:
        return "cpu"
    try:
        import torch

        return torch.cuda.get_device_properties(comm.device).gcnArchName.split(":")[0]
    except Exception:
        return "unknown"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _benchmark_worker_entry(result_queue, init_method: str, kwargs: Dict[str, Any]) -> None:
    """Spawned child: fresh HIP context, own process group, one row back to the parent."""
    os.environ["DDLB_CHILD_INIT_METHOD"] = init_method
    row = None
    try:
        row = run_single(**kwargs)
    except Exception as e:
        row = {"error": f"{type(e).__name__}: {e}", "valid": False}
    finally:
        try:
            from ddlb_amd.communicator import Communicator

            Communicator.reset()
        except Exception:
            pass
        result_queue.put(row)


class PrimitiveBenchmarkRunner:
    """Run every implementation config of one shape, each in its own spawned process."""

    ALLOWED_PRIMITIVES = {"tp_columnwise", "tp_rowwise"}
    _child_counter = 0

    def __init__(self, primitive: str, m: int, n: int, k: int, implementations: List[str],
                 dtype: str = "float32", validate: bool = True, num_iterations: int = 5,
                 num_warmups: int = 2, implementation_options: Optional[Dict[str, Dict]] = None,
                 output_csv: Optional[str] = None, time_measurement_backend: str = "cpu_clock",
                 barrier_at_each_iteration: bool = True, profile_iterations: int = 5,
                 child_timeout_s: float = 1800.0, resume: bool = False, isolate: bool = True,
                 validate_every_iteration: bool = False, pmc=None,
                 pmc_dir: str = "results/pmc"):
        if primitive not in self.ALLOWED_PRIMITIVES:
            raise ValueError(f"Unknown primitive: {primitive}")
        from ddlb_amd.utils import pmc as pmc_mod

        self.pmc = pmc_mod.parse(pmc)
        if self.pmc:
            pmc_mod.check_limits(self.pmc)  # before any launch: an over-full pass hangs
        self.pmc_dir = pmc_dir
        self.primitive = primitive
        self.m, self.n, self.k = int(m), int(n), int(k)
        self.implementations = list(implementations)
        self.dtype = dtype
        self.validate = validate
        self.num_iterations = int(num_iterations)
        self.num_warmups = int(num_warmups)
        self.implementation_options = implementation_options or {}
        self.output_csv = output_csv
        self.time_measurement_backend = time_measurement_backend
        self.barrier_at_each_iteration = barrier_at_each_iteration
        self.profile_iterations = int(profile_iterations)
        self.child_timeout_s = float(child_timeout_s)
        self.resume = resume
        self.isolate = isolate
        self.validate_every_iteration = validate_every_iteration

    # ------------------------------------------------------------------ helpers
    def _kwargs(self, impl_id: str) -> Dict[str, Any]:
        return dict(primitive=self.primitive, impl_id=impl_id, m=self.m, n=self.n, k=self.k,
                    dtype=self.dtype, num_warmups=self.num_warmups,
                    num_iterations=self.num_iterations,
                    impl_opts=dict(self.implementation_options.get(impl_id, {})),
                    validate=self.validate,
                    time_measurement_backend=self.time_measurement_backend,
                    barrier_at_each_iteration=self.barrier_at_each_iteration,
                    profile_iterations=self.profile_iterations,
                    validate_every_iteration=self.validate_every_iteration)

    _store = None  # parent-level TCPStore (world > 1): rank 0 publishes each child's port

    def _next_init_method(self) -> str:
        """Rendezvous of the next child process group. Rank 0 binds a currently free port and,
        when there are several ranks, publishes it through a small TCPStore the parent
        processes share (created once at the base port; no GPU involved), so every rank's
        child dials the same, actually free port (a fixed port sequence collided with ephemeral
        ports of earlier children's sockets: EADDRINUSE)."""
        idx = PrimitiveBenchmarkRunner._child_counter
        PrimitiveBenchmarkRunner._child_counter += 1
        rank, world = get_rank(), get_world_size()
        port = _free_port() if rank == 0 else 0
        if world > 1:
            import datetime

            from torch.distributed import TCPStore

            if PrimitiveBenchmarkRunner._store is None:
                PrimitiveBenchmarkRunner._store = TCPStore(
                    get_master_addr(), get_master_port(), world, rank == 0,
                    timeout=datetime.timedelta(seconds=self.child_timeout_s))
            key = f"ddlb_child_port_{idx}"
            if rank == 0:
                PrimitiveBenchmarkRunner._store.set(key, str(port))
            else:
                port = int(PrimitiveBenchmarkRunner._store.get(key).decode())
        return f"tcp://{get_master_addr()}:{port}"

    def _done_keys(self) -> set:
        keys = set()
        if not (self.resume and self.output_csv and os.path.exists(self.output_csv)):
            return keys
        with open(self.output_csv, newline="") as f:
            for r in csv.DictReader(f):
                keys.add((r.get("spec", ""), r.get("m"), r.get("n"), r.get("k"), r.get("dtype"),
                          r.get("world_size")))
        return keys

    def _run_child_pmc(self, impl_id: str, init: str, kwargs: Dict[str, Any]) -> Dict[str, Any]:
        """The child as a fresh program under ``rocprofv3 --pmc ... --selected-regions``: the
        counters cover the profiler window (``profile_iterations`` run() calls); their
        per-kernel means come back in the row's ``pmc`` column."""
        from ddlb_amd.utils import pmc as pmc_mod

        tag = f"{self.primitive}_{self.m}x{self.n}x{self.k}_{impl_id}_rank{get_rank()}"
        out_dir = os.path.abspath(os.path.join(self.pmc_dir, tag))
        os.makedirs(out_dir, exist_ok=True)
        jin, jout = os.path.join(out_dir, "kwargs.json"), os.path.join(out_dir, "row.json")
        with open(jin, "w") as f:
            json.dump(kwargs, f)
        if os.path.exists(jout):
            os.remove(jout)
        env = dict(os.environ, DDLB_CHILD_INIT_METHOD=init)
        cmd = pmc_mod.rocprof_cmd(self.pmc, out_dir) + [
            sys.executable, "-m", "ddlb_amd.benchmark", "--worker", jin, jout]
        proc = subprocess.Popen(cmd, env=env)
        try:
            proc.wait(timeout=self.child_timeout_s)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
            return {"valid": False, "error": f"child timed out after {self.child_timeout_s:.0f}s",
                    "pmc": ""}
        if not os.path.exists(jout):
            return {"valid": False, "error": f"profiled child exited with code {proc.returncode}",
                    "pmc": ""}
        with open(jout) as f:
            row = json.load(f)
        try:
            row["pmc"] = json.dumps(pmc_mod.summarize(out_dir, top=8), sort_keys=True)
        except Exception as e:  # the measurement stands without counters
            row["pmc"] = f"unavailable: {type(e).__name__}: {e}"
        return row

    def _run_child(self, impl_id: str) -> Dict[str, Any]:
        init = self._next_init_method()
        kwargs = self._kwargs(impl_id)
        if self.pmc:
            return self._run_child_pmc(impl_id, init, kwargs)
        if not self.isolate:
            os.environ["DDLB_CHILD_INIT_METHOD"] = init
            try:
                return run_single(**kwargs)
            finally:
                from ddlb_amd.communicator import Communicator

                Communicator.reset()
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        proc = ctx.Process(target=_benchmark_worker_entry, args=(q, init, kwargs))
        proc.start()
        row = None
        deadline = time.monotonic() + self.child_timeout_s
        while row is None:
            try:
                row = q.get(timeout=1.0)
            except _queue.Empty:
                if not proc.is_alive():
                    try:
                        row = q.get(timeout=2.0)
                    except _queue.Empty:
                        row = {"valid": False,
                               "error": f"child exited with code {proc.exitcode} before reporting"}
                elif time.monotonic() > deadline:
                    proc.terminate()
                    proc.join(10)
                    if proc.is_alive():
                        proc.kill()
                    row = {"valid": False,
                           "error": f"child timed out after {self.child_timeout_s:.0f}s"}
        proc.join(30)
        if proc.is_alive():
            proc.kill()
        return row

    def _complete_row(self, impl_id: str, row: Dict[str, Any]) -> Dict[str, Any]:
        opts = self.implementation_options.get(impl_id, {})
        base = dict(implementation=opts.get("implementation", impl_id), m=self.m, n=self.n,
                    k=self.k, dtype=self.dtype, world_size=get_world_size(),
                    hostname=socket.gethostname(),
                    time_measurement_backend=self.time_measurement_backend,
                    barrier_at_each_iteration=self.barrier_at_each_iteration, option="")
        for key, v in base.items():
            row.setdefault(key, v)
        for key in ("mean_time (ms)", "std_time", "min_time", "max_time",
                    "Throughput (TFLOPS)", "Throughput std (TFLOPS)"):
            row.setdefault(key, 0.0)
        row.setdefault("gpu_arch", "")
        row.setdefault("error", "")
        if self.validate:
            row.setdefault("valid", False)
        row["spec"] = _spec_key(opts)
        return order_row(row)

    def _append_csv(self, path: str, row: Dict[str, Any]) -> None:
        cols = [c for c in CSV_COLUMNS if c != "valid" or self.validate] + EXTRA_COLUMNS + ["spec"]
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        write_header = not os.path.exists(path) or os.path.getsize(path) == 0
        with open(path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols, extrasaction="ignore",
                               quoting=csv.QUOTE_MINIMAL)
            if write_header:
                w.writeheader()
            w.writerow(row)

    # ------------------------------------------------------------------ main
    def run(self):
        import pandas as pd

        rank = get_rank()
        done = self._done_keys()
        results: List[Dict[str, Any]] = []
        try:
            from tqdm import tqdm
        except ImportError:  # pragma: no cover
            tqdm = None
        it = self.implementations
        if rank == 0 and tqdm is not None and os.environ.get("DDLB_PROGRESS", "1") == "1":
            it = tqdm(it, desc="Running benchmarks", position=0)
        for impl_id in it:
            opts = self.implementation_options.get(impl_id, {})
            key = (_spec_key(opts), str(self.m), str(self.n), str(self.k), self.dtype,
                   str(get_world_size()))
            if key in done:
                if rank == 0:
                    print(f"Skipping {impl_id} (already in {self.output_csv})")
                continue
            if rank == 0:
                print(f"Running benchmark for {impl_id} with options {opts}")
            row = self._complete_row(impl_id, self._run_child(impl_id))
            if rank == 0:
                shown = {k: v for k, v in row.items() if k != "spec"}
                print(pd.DataFrame([shown]).to_string(index=False))
                if self.output_csv:
                    self._append_csv(self.output_csv, row)
            results.append(row)
        return pd.DataFrame(results)

    def plot_results(self, results=None, path: Optional[str] = None) -> Optional[str]:
        """Bar chart of mean time +- std (``ddlb/benchmark.py:391-425``); saved to ``path``."""
        if results is None:
            results = self.run()
        try:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except ImportError:
            print("matplotlib is not installed; skipping plot")
            return None
        fig = plt.figure(figsize=(12, 6))
        plt.bar(list(results["implementation"]), results["mean_time (ms)"],
                yerr=results["std_time"], capsize=5)
        plt.title(f"{self.primitive.upper()} Benchmark\nSize: ({self.m},{self.n},{self.k}), "
                  f"Dtype: {self.dtype}")
        plt.ylabel("Time (ms)")
        plt.xticks(rotation=45, ha="right")
        plt.tight_layout()
        path = path or f"results/{self.primitive}_{self.m}x{self.k}x{self.n}_{self.dtype}.png"
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        fig.savefig(path)
        plt.close(fig)
        return path


def _worker_main(argv: List[str]) -> int:
    """``python -m ddlb_amd.benchmark --worker KWARGS.json ROW.json``: one benchmark child as a
    standalone program (the form a profiler launcher can wrap)."""
    if len(argv) != 3 or argv[0] != "--worker":
        raise SystemExit("usage: python -m ddlb_amd.benchmark --worker KWARGS.json ROW.json")
    with open(argv[1]) as f:
        kwargs = json.load(f)
    try:
        row = run_single(**kwargs)
    except Exception as e:
        row = {"error": f"{type(e).__name__}: {e}", "valid": False}
    finally:
        try:
            from ddlb_amd.communicator import Communicator

            Communicator.reset()
        except Exception:
            pass
    with open(argv[2], "w") as f:
        json.dump(row, f, default=str)
    return 0


if __name__ == "__main__":
    sys.exit(_worker_main(sys.argv[1:]))
