"""Command-line and programmatic entry points.

Parity: ``ddlb/cli/benchmark.py:120-316`` (``run_benchmark(config)`` and ``main()``).
Same flags (``--primitive -m -n -k --dtype --num-iterations --num-warmups --output-csv
--impl``), same JSON schema and impl-spec grammar. Fixes / additions:

* ``--primitive`` accepts ``tp_rowwise`` (the reference's argparse only allows
  ``tp_columnwise`` although its README shows a rowwise example);
* ``--no-validate`` (the reference's ``--validate`` is ``store_true`` with default True, so it
  can never be turned off), ``--time-measurement-backend``, ``--no-barrier``,
  ``--profile-iterations``, ``--child-timeout``, ``--resume``, ``--no-isolate``,
  ``--validate-every-iteration``, ``--config`` (JSON file) and ``--plot``.
"""

from __future__ import annotations

import argparse
import json
import os
from datetime import datetime
from typing import Any, Dict, List, Optional

from ddlb_amd.cli.config import build_impl_table, generate_config_combinations, \
    normalize_benchmark_config, parse_impl_spec, parse_int_list
from ddlb_amd.envs import get_rank, get_world_size
from ddlb_amd.utils.stats import SUMMARY_COLUMNS


def resolve_csv_path(output_csv: Optional[str], primitive: str, m: List[int], n: List[int],
                     k: List[int], dtype: str, stamp: Optional[str] = None) -> str:
    """``{timestamp}`` substitution or ``results/<prim>_<m>x<k>x<n>_<dtype>_<ts>.csv`` (:179-188)."""
    stamp = stamp or datetime.now().strftime("%Y%m%d_%H%M%S")
    if output_csv and str(output_csv).strip():
        return str(output_csv).replace("{timestamp}", stamp)
    label = f"{m[0]}x{k[0]}x{n[0]}" if m and n and k else "shapes"
    return f"results/{primitive}_{label}_{dtype}_{stamp}.csv"


def run_benchmark(config: Dict[str, Any], isolate: bool = True, plot: bool = False):
    """Run every (shape x expanded implementation config); returns the results DataFrame."""
    import itertools

    import pandas as pd

    from ddlb_amd.benchmark import PrimitiveBenchmarkRunner

    bench = normalize_benchmark_config(config)
    rank, world = get_rank(), get_world_size()
    primitive = bench["primitive"]
    expanded = generate_config_combinations(bench["implementations"])
    shapes = list(itertools.product(bench["m"], bench["n"], bench["k"]))
    ids, impl_options = build_impl_table(expanded)
    csv_path = resolve_csv_path(bench["output_csv"], primitive, bench["m"], bench["n"],
                                bench["k"], bench["dtype"])
    if rank == 0:
        print(f"Running {primitive} benchmark with {world} processes")
        print(f"Number of shapes: {len(shapes)}")
        print("Shapes:")
        for mm, nn, kk in shapes:
            print(f"  ({mm}, {nn}, {kk})")
        print("\nConfigurations:")
        for impl_id in ids:
            print(f"  {impl_id}: {impl_options[impl_id]}")
    frames = []
    for mm, nn, kk in shapes:
        if rank == 0:
            print(f"\n--- Running shape ({mm}, {nn}, {kk}) ---")
        runner = PrimitiveBenchmarkRunner(
            primitive=primitive, m=mm, n=nn, k=kk, implementations=ids, dtype=bench["dtype"],
            validate=bool(bench["validate"]), num_iterations=bench["num_iterations"],
            num_warmups=bench["num_warmups"], implementation_options=impl_options,
            output_csv=csv_path, time_measurement_backend=bench["time_measurement_backend"],
            barrier_at_each_iteration=bool(bench["barrier_at_each_iteration"]),
            profile_iterations=int(bench["profile_iterations"]),
            child_timeout_s=float(bench["child_timeout_s"]), resume=bool(bench["resume"]),
            isolate=isolate, validate_every_iteration=bool(bench.get("validate_every_iteration",
                                                                     False)),
            pmc=bench.get("pmc"), pmc_dir=bench.get("pmc_dir") or "results/pmc")
        df = runner.run()
        if plot and rank == 0 and len(df):
            runner.plot_results(df, path=os.path.splitext(csv_path)[0] + f"_{mm}x{kk}x{nn}.png")
        frames.append(df)
    results = pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()
    if rank == 0 and len(results):
        print("\nBenchmark Results:")
        results["config"] = results["implementation"]
        cols = [c for c in SUMMARY_COLUMNS if c in results.columns]
        with pd.option_context("display.max_columns", None, "display.width", None,
                               "display.max_colwidth", None):
            print(results[cols].to_string())
        print(f"\nCSV: {csv_path}")
    return results


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="ddlb_amd",
                                description="MI355X distributed-GEMM benchmark (DDLB-compatible)")
    p.add_argument("--config", help="JSON config file (scripts/config.json format); "
                                    "other flags are ignored when given")
    p.add_argument("--primitive", choices=["tp_columnwise", "tp_rowwise"])
    p.add_argument("-m", "--m", help="comma list of m sizes")
    p.add_argument("-n", "--n", help="comma list of n sizes")
    p.add_argument("-k", "--k", help="comma list of k sizes")
    p.add_argument("--dtype", default="float16")
    p.add_argument("--validate", dest="validate", action="store_true", default=True)
    p.add_argument("--no-validate", dest="validate", action="store_false")
    p.add_argument("--num-iterations", type=int, default=50)
    p.add_argument("--num-warmups", type=int, default=5)
    p.add_argument("--output-csv", default=None, help="CSV path; supports {timestamp}")
    p.add_argument("--impl", action="append",
                   help="name;key=value[,value];flag  (repeat for more base configs)")
    p.add_argument("--time-measurement-backend", default="cpu_clock",
                   choices=["cpu_clock", "cuda_event", "hip_event"])
    p.add_argument("--barrier", dest="barrier", action="store_true", default=True)
    p.add_argument("--no-barrier", dest="barrier", action="store_false")
    p.add_argument("--profile-iterations", type=int, default=5)
    p.add_argument("--child-timeout", type=float, default=1800.0)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--no-isolate", action="store_true",
                   help="run configs in this process instead of spawned children")
    p.add_argument("--validate-every-iteration", action="store_true",
                   help="debug/race screen: validate every timed iteration")
    p.add_argument("--plot", action="store_true", help="save a bar chart next to the CSV")
    p.add_argument("--pmc", default=None,
                   help="comma list of hardware counters (or 'default') collected by rocprofv3 "
                        "over the 5-iteration profiler window of every child; per-kernel means "
                        "land in the CSV's pmc column (one pass: <= 8 SQ, 4 TCC, 2 GRBM, ...)")
    p.add_argument("--pmc-dir", default="results/pmc", help="rocprofv3 output directory root")
    return p


def main(argv: Optional[List[str]] = None) -> None:
    args = build_parser().parse_args(argv)
    if args.config:
        with open(args.config) as f:
            config = json.load(f)
        run_benchmark(config, isolate=not args.no_isolate, plot=args.plot)
        return
    missing = [f for f in ("primitive", "m", "n", "k", "impl") if not getattr(args, f)]
    if missing:
        raise SystemExit(f"missing required arguments: {', '.join('--' + x for x in missing)}")
    impls: Dict[str, List[Dict[str, Any]]] = {}
    for spec in args.impl:
        name, opts = parse_impl_spec(spec)
        impls.setdefault(name, []).append(opts)
    config = {"benchmark": {
        "primitive": args.primitive, "m": parse_int_list(args.m), "n": parse_int_list(args.n),
        "k": parse_int_list(args.k), "dtype": args.dtype, "validate": args.validate,
        "num_iterations": args.num_iterations, "num_warmups": args.num_warmups,
        "output_csv": args.output_csv, "implementations": impls,
        "time_measurement_backend": args.time_measurement_backend,
        "barrier_at_each_iteration": args.barrier, "profile_iterations": args.profile_iterations,
        "child_timeout_s": args.child_timeout, "resume": args.resume,
        "validate_every_iteration": args.validate_every_iteration,
        "pmc": args.pmc, "pmc_dir": args.pmc_dir,
    }}
    run_benchmark(config, isolate=not args.no_isolate, plot=args.plot)


if __name__ == "__main__":
    main()
