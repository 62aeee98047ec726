"""Benchmark configuration: impl-spec mini-language, cartesian expansion, JSON schema.

Parity with ``ddlb/cli/benchmark.py``:

* ``infer_scalar``          ~ ``_infer_scalar``  (:14-32)
* ``parse_value_list``      ~ ``_parse_value_list`` (:35-46)
* ``parse_int_list``        ~ ``_parse_int_list`` (:49-52)
* ``parse_impl_spec``       ~ ``_parse_impl_spec`` (:55-83)  grammar ``name;key=v1,v2;flag``
* ``generate_config_combinations`` (:85-118) cartesian product *within* a base config
* ``normalize_benchmark_config`` fills the defaults ``run_benchmark`` reads (:131-145)

One deliberate fix: the reference intends a leading-zero token such as ``08`` to stay a
string but its float fallback turns it into ``8.0``. Here ``08`` stays
``"08"``; ``0.5`` is still a float.
"""

from __future__ import annotations

import itertools
from typing import Any, Dict, List, Mapping, Tuple

DEFAULTS: Dict[str, Any] = {
    "dtype": "float32",           # base-class default (tp_columnwise.py:32)
    "validate": True,
    "num_iterations": 5,          # runner default (benchmark.py:278)
    "num_warmups": 2,
    "time_measurement_backend": "cpu_clock",
    "barrier_at_each_iteration": True,
    "output_csv": None,
    "profile_iterations": 5,      # reference hard-codes the 5-iteration profiler window
    "child_timeout_s": 1800.0,
    "pmc": None,                  # opt-in rocprofv3 counters over the profiler window (utils/pmc)
    "pmc_dir": "results/pmc",
    "resume": False,
}

TIME_BACKENDS = ("cpu_clock", "cuda_event", "hip_event")
PRIMITIVES = ("tp_columnwise", "tp_rowwise")


def infer_scalar(value: str) -> Any:
    """bool -> int -> float -> str, keeping leading-zero tokens (``"08"``) as strings."""
    v = value.strip()
    low = v.lower()
    if low in ("true", "false"):
        return low == "true"
    leading_zero = len(v) > 1 and v[0] == "0" and v[1] != "." and v.lstrip("0") != ""
    if leading_zero:
        return v
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v)
    except ValueError:
        return v


def parse_value_list(v: str) -> Any:
    """Comma list -> list of inferred scalars; a single token -> scalar; empty -> ``""``."""
    parts = [p.strip() for p in (v or "").split(",") if p.strip()]
    if not parts:
        return ""
    if len(parts) == 1:
        return infer_scalar(parts[0])
    return [infer_scalar(p) for p in parts]


def parse_int_list(v: Any) -> List[int]:
    if isinstance(v, (list, tuple)):
        return [int(x) for x in v]
    return [int(x) for x in str(v).split(",") if x.strip()]


def parse_impl_spec(spec: str) -> Tuple[str, Dict[str, Any]]:
    """Parse ``name;key=value[,value];flag`` into ``(name, options)``."""
    if spec is None:
        raise ValueError("Empty implementation spec")
    tokens = [t for t in str(spec).split(";") if t.strip()]
    if not tokens:
        raise ValueError("Invalid implementation spec: empty")
    name = tokens[0].strip()
    options: Dict[str, Any] = {}
    for tok in tokens[1:]:
        if "=" not in tok:
            key = tok.strip()
            if key:
                options[key] = True
            continue
        key, val = tok.split("=", 1)
        key = key.strip()
        if key:
            options[key] = parse_value_list(val.strip())
    return name, options


def generate_config_combinations(
        config: Mapping[str, List[Mapping[str, Any]]]) -> Dict[str, List[Dict[str, Any]]]:
    """Expand every list-valued option of each base config by cartesian product."""
    expanded: Dict[str, List[Dict[str, Any]]] = {}
    for impl_name, base_configs in config.items():
        if isinstance(base_configs, Mapping):
            base_configs = [base_configs]
        out: List[Dict[str, Any]] = []
        for base in base_configs:
            list_params = {k: v for k, v in base.items() if isinstance(v, list)}
            if not list_params:
                out.append(dict(base))
                continue
            names = list(list_params)
            for combo in itertools.product(*(list_params[n] for n in names)):
                cfg = dict(base)
                cfg.update(zip(names, combo))
                out.append(cfg)
        expanded[impl_name] = out
    return expanded


def to_list(x: Any) -> List[Any]:
    return list(x) if isinstance(x, (list, tuple)) else [x]


def normalize_benchmark_config(config: Mapping[str, Any]) -> Dict[str, Any]:
    """Validate a ``{"benchmark": {...}}`` dict and fill defaults. Returns the inner dict."""
    if "benchmark" not in config:
        raise ValueError("config must have a top-level 'benchmark' key")
    bench = dict(config["benchmark"])
    for key in ("primitive", "m", "n", "k", "implementations"):
        if key not in bench:
            raise ValueError(f"benchmark config is missing '{key}'")
    if bench["primitive"] not in PRIMITIVES:
        raise ValueError(f"Unknown primitive: {bench['primitive']} (allowed: {PRIMITIVES})")
    for key, default in DEFAULTS.items():
        bench.setdefault(key, default)
    if bench["time_measurement_backend"] not in TIME_BACKENDS:
        raise ValueError(f"Unknown time_measurement_backend: {bench['time_measurement_backend']}")
    if bench["time_measurement_backend"] == "hip_event":
        bench["time_measurement_backend"] = "cuda_event"
    for key in ("m", "n", "k"):
        bench[key] = [int(v) for v in to_list(bench[key])]
    impls = bench["implementations"]
    if not isinstance(impls, Mapping) or not impls:
        raise ValueError("'implementations' must be a non-empty mapping name -> [configs]")
    return bench


def build_impl_table(expanded: Mapping[str, List[Dict[str, Any]]]
                     ) -> Tuple[List[str], Dict[str, Dict[str, Any]]]:
    """``impl_id = "<name>_<i>"`` and ``options = {'implementation': name, **opts}`` (:166-177)."""
    ids: List[str] = []
    options: Dict[str, Dict[str, Any]] = {}
    for name, cfgs in expanded.items():
        for i, opts in enumerate(cfgs):
            impl_id = f"{name}_{i}"
            ids.append(impl_id)
            options[impl_id] = {"implementation": name, **opts}
    return ids, options


def base_impl_name(impl_id: str) -> str:
    """Strip the ``_<idx>`` suffix (``ddlb/benchmark.py:70-73``)."""
    head, sep, tail = impl_id.rpartition("_")
    return head if sep and tail.isdigit() else impl_id
