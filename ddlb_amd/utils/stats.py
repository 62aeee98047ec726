"""Timing statistics and the result-row schema.

Parity: ``ddlb/benchmark.py:206-245``.

* ``mean_time (ms)`` = mean of the MAX-over-ranks per-iteration times, ``std_time`` = population
  std (``np.std``), min / max;
* per-iteration TFLOPS = ``(2*m*n*k / 1e9) / t_ms``; the row carries their mean and std.

``CSV_COLUMNS`` is the reference column order; native extras are appended at the end only
(SURVEY.md §5.5), so reference CSV consumers keep working.
"""

from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

CSV_COLUMNS: List[str] = [
    "implementation", "mean_time (ms)", "std_time", "min_time", "max_time", "m", "n", "k",
    "dtype", "Throughput (TFLOPS)", "Throughput std (TFLOPS)", "world_size", "hostname",
    "time_measurement_backend", "barrier_at_each_iteration", "option", "valid",
]
EXTRA_COLUMNS: List[str] = ["per_gpu_tflops", "algbw_GBps", "gpu_arch", "error", "pmc"]

SUMMARY_COLUMNS = ["m", "n", "k", "config", "Throughput (TFLOPS)", "Throughput std (TFLOPS)",
                   "mean_time (ms)", "std_time", "min_time", "max_time"]


def summarize(times_ms: Sequence[float], m: int, n: int, k: int) -> Dict[str, float]:
    t = np.asarray(list(times_ms), dtype=np.float64)
    thr_const = (2.0 * m * n * k) / 1e9
    thr = thr_const / t[t > 0] if t.size else np.zeros(0)
    return {
        "mean_time (ms)": float(t.mean()) if t.size else 0.0,
        "std_time": float(t.std()) if t.size else 0.0,
        "min_time": float(t.min()) if t.size else 0.0,
        "max_time": float(t.max()) if t.size else 0.0,
        "Throughput (TFLOPS)": float(thr.mean()) if thr.size else 0.0,
        "Throughput std (TFLOPS)": float(thr.std()) if thr.size else 0.0,
    }


_ESZ = {"float32": 4, "float16": 2, "bfloat16": 2, "float8_e4m3fn": 1, "float64": 8,
        "int32": 4, "int64": 8}


def derived_metrics(primitive: str, base_impl: str, size: str, m: int, n: int, k: int,
                    dtype: str, world: int, mean_ms: float) -> Dict[str, float]:
    """Append-only extras that undo the harness formula's per-primitive meaning:

    * ``per_gpu_tflops``: tp_columnwise's harness number already is per GPU (every rank does
      2mnk); tp_rowwise's and sharded compute_only's are aggregates, so they are divided by d.
    * ``algbw_GBps``: collective payload / time, NCCL's "algorithm bandwidth" convention — the
      gathered [m, k] input for tp_columnwise, the reduce-scattered [m, n] output for
      tp_rowwise; 0 for compute_only.
    """
    if mean_ms <= 0:
        return {"per_gpu_tflops": 0.0, "algbw_GBps": 0.0}
    d = max(int(world), 1)
    tflops = 2.0 * m * n * k / (mean_ms * 1e9)
    esz = _ESZ.get(dtype, 2)
    if base_impl == "compute_only":
        per_gpu = tflops / d if size == "sharded" else tflops
        payload = 0
    elif primitive == "tp_rowwise":
        per_gpu = tflops / d
        payload = m * n * (2 if esz == 1 else esz)  # fp8 GEMMs emit bf16
    else:
        per_gpu = tflops
        payload = m * k * esz
    return {"per_gpu_tflops": per_gpu,
            "algbw_GBps": (payload / (mean_ms * 1e-3) / 1e9) if d > 1 else 0.0}


def impl_label(base_impl: str, options: Dict, default_keys: Sequence[str]) -> str:
    """``"<impl> (k=v, ...)"`` in DEFAULT_OPTIONS order, ``size`` excluded (:106-115)."""
    shown = [(k, options[k]) for k in default_keys if k in options and k != "size"]
    if not shown:
        return base_impl
    return f"{base_impl} (" + ", ".join(f"{k}={v}" for k, v in shown) + ")"


def option_string(options: Dict, default_keys: Sequence[str]) -> str:
    return ", ".join(f"{k}={options[k]}" for k in default_keys if k in options and k != "size")


def order_row(row: Dict) -> Dict:
    """Reference columns first (``valid`` only when present), extras last."""
    out = {c: row[c] for c in CSV_COLUMNS if c in row}
    for c in EXTRA_COLUMNS:
        if c in row:
            out[c] = row[c]
    for c, v in row.items():
        if c not in out:
            out[c] = v
    return out
