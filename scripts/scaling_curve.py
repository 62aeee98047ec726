"""Scaling curve at 1/2/4/8 GPUs -> BASELINE.md-style markdown table.

Two sources:

  * run:  launch ``bench.py`` once per world size on this node (world 1 directly, N > 1 through
    ``torch.distributed.run`` on 127.0.0.1, one rank per GPU), keep each run's JSON line::

        python scripts/scaling_curve.py --gpus 1,2,4,8 --steps 50 --warmup 10 [-- bench args]

  * render: tabulate result lines that already exist (bench.py JSON lines, a driver SCALE file,
    or DDLB CSVs written by the CLI runner at several world sizes)::

        python scripts/scaling_curve.py --from results/scale.jsonl results/col_*.csv

Efficiency is the reference's reading of its own harness: weak scaling (bench.py: per-GPU work
fixed) -> ``value(N) / (N * value(1) / 1)``; strong scaling (fixed total work) -> ``t(1) / (N t(N))``.
The table's rows are keyed by (label, world size); the best row per key is kept.
"""

from __future__ import annotations

import argparse
import csv
import json
import os
import socket
import subprocess
import sys
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def bench_command(n: int, steps: int, warmup: int, extra: List[str], port: int) -> List[str]:
    """The driver's launch contract for bench.py (one rank per GPU, rendezvous on 127.0.0.1)."""
    tail = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps),
            "--warmup", str(warmup)] + list(extra)
    if n == 1:
        return [sys.executable] + tail
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port)] + tail


def parse_json_lines(text: str) -> List[dict]:
    rows = []
    for line in text.splitlines():
        line = line.strip()
        if not (line.startswith("{") and line.endswith("}")):
            continue
        try:
            obj = json.loads(line)
        except json.JSONDecodeError:
            continue
        if isinstance(obj, dict) and "n_gpus" in obj and "ms_per_step" in obj:
            rows.append(obj)
        elif isinstance(obj, dict) and isinstance(obj.get("runs"), list):  # {"runs": [...]}
            rows += [r for r in obj["runs"] if isinstance(r, dict) and "n_gpus" in r]
    return rows


def _bench_row(obj: dict) -> dict:
    cfg = obj.get("config", {})
    return {"label": f"{cfg.get('model', obj.get('metric', '?'))} [{obj.get('dtype', '?')}]",
            "n": int(obj["n_gpus"]), "ms": float(obj["ms_per_step"]),
            "value": float(obj["value"]), "unit": obj.get("unit", ""),
            "scaling": obj.get("scaling", "weak"),
            "algorithm": cfg.get("algorithm", cfg.get("parallelism", "")),
            "valid": obj.get("valid", True)}


def parse_csv(path: str) -> List[dict]:
    """DDLB CSV rows (CLI runner): Throughput is the harness number; scaling is strong."""
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if r.get("error") or not r.get("mean_time (ms)"):
                continue
            impl = r["implementation"].split(" (")[0]
            rows.append({"label": f"{impl} m={r['m']} n={r['n']} k={r['k']} [{r['dtype']}]",
                         "n": int(r["world_size"]), "ms": float(r["mean_time (ms)"]),
                         "value": float(r["Throughput (TFLOPS)"]), "unit": "TFLOP/s",
                         "scaling": "strong", "algorithm": r.get("option", "")[:60],
                         "valid": r.get("valid", "True") in ("True", "true", "1", "")})
    return rows


def best_per_key(rows: List[dict]) -> Dict[str, Dict[int, dict]]:
    out: Dict[str, Dict[int, dict]] = {}
    for r in rows:
        if not r["valid"]:
            continue
        slot = out.setdefault(r["label"], {})
        if r["n"] not in slot or r["ms"] < slot[r["n"]]["ms"]:
            slot[r["n"]] = r
    return out


def efficiency(r: dict, base: Optional[dict]) -> Optional[float]:
    if base is None:
        return None
    n_ratio = r["n"] / base["n"]
    if r["scaling"] == "weak":
        return r["value"] / (n_ratio * base["value"])
    return base["ms"] / (n_ratio * r["ms"])


def render(rows: List[dict]) -> str:
    lines = []
    for label, by_n in sorted(best_per_key(rows).items()):
        base = by_n[min(by_n)]
        unit = base["unit"] or "TFLOP/s"
        lines += [f"### {label} ({base['scaling']} scaling)", "",
                  f"| GPUs | ms/iter | {unit} (whole job) | {unit} per GPU | efficiency vs "
                  f"{base['n']} GPU | algorithm |",
                  "|---|---|---|---|---|---|"]
        for n in sorted(by_n):
            r = by_n[n]
            eff = efficiency(r, base)
            lines.append(f"| {n} | {r['ms']:.4f} | {r['value']:.1f} | {r['value'] / n:.1f} | "
                         f"{'-' if eff is None else f'{100 * eff:.1f} %'} | {r['algorithm']} |")
        lines.append("")
    return "\n".join(lines)


def load(paths: List[str]) -> List[dict]:
    rows: List[dict] = []
    for p in paths:
        if p.endswith(".csv"):
            rows += parse_csv(p)
        else:
            with open(p) as f:
                rows += [_bench_row(o) for o in parse_json_lines(f.read())]
    return rows


def run(gpus: List[int], steps: int, warmup: int, extra: List[str], timeout: float) -> List[dict]:
    rows = []
    for n in gpus:
        cmd = bench_command(n, steps, warmup, extra, _free_port())
        print(f"[scaling] N={n}: {' '.join(cmd)}", file=sys.stderr, flush=True)
        try:
            proc = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
        except subprocess.TimeoutExpired:
            print(f"[scaling] N={n}: timed out after {timeout:.0f} s", file=sys.stderr)
            continue
        found = parse_json_lines(proc.stdout)
        if proc.returncode != 0 or not found:
            print(f"[scaling] N={n}: rc={proc.returncode}\n{proc.stderr[-2000:]}", file=sys.stderr)
            continue
        print(json.dumps(found[-1]), flush=True)
        rows.append(_bench_row(found[-1]))
    return rows


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    extra: List[str] = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", default="1,2,4,8", help="comma list of world sizes to run")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--timeout", type=float, default=1800.0, help="per world size (s)")
    p.add_argument("--from", dest="sources", nargs="+", default=None,
                   help="render existing JSON-line / CSV results instead of running")
    p.add_argument("--out", default=None, help="also write the markdown table here")
    a = p.parse_args(argv)
    if a.sources:
        rows = load(a.sources)
    else:
        rows = run([int(x) for x in a.gpus.split(",") if x], a.steps, a.warmup, extra, a.timeout)
    table = render(rows)
    print(table)
    if a.out:
        with open(a.out, "w") as f:
            f.write(table + "\n")
    return 0 if rows else 1


if __name__ == "__main__":
    sys.exit(main())
