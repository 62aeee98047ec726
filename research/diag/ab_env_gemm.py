"""A/B of an environment knob of the native GEMM (read once per process by the launcher): each
variant runs ``scripts/bench_gemm.py`` in its own process, variants interleaved over rounds, the
native ``auto`` row's median per variant and shape reported (one box, one call). The value
``unset`` runs with the knob absent.

    python research/diag/ab_env_gemm.py --knob DDLB_PT4_CAUX --values 18,16,19,2 --shapes 0,6 --rounds 3
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--knob", required=True)
    p.add_argument("--values", required=True)
    p.add_argument("--shapes", default="0")
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--modes", default="auto")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--json", default=None)
    a = p.parse_args()
    vals = a.values.split(",")
    res = {}
    for rnd in range(a.rounds):
        for v in vals:
            out = os.path.join("/tmp", f"ab_{os.getpid()}_{rnd}_{v}.json")
            env = dict(os.environ)
            if v == "unset":  # the knob absent (knobs read as "set or not")
                env.pop(a.knob, None)
            else:
                env[a.knob] = v
            cmd = [sys.executable, os.path.join(ROOT, "scripts", "bench_gemm.py"), "--shapes",
                   a.shapes, "--tiles", "auto", "--modes", a.modes, "--dtype", a.dtype,
                   "--rounds", "3", "--json", out]
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
            if r.returncode != 0:
                print(f"{a.knob}={v}: failed\n{r.stderr[-2000:]}", flush=True)
                return 1
            for row in json.load(open(out)):
                key = f"{row['M']}x{row['N']}x{row['K']}"
                for name, d in row["variants"].items():
                    res.setdefault((key, name, v), []).append(d["ms_median"])
            os.remove(out)
            print(f"round {rnd} {a.knob}={v} done", flush=True)
    table = {}
    for (key, name, v), ts in sorted(res.items()):
        med = statistics.median(ts)
        table.setdefault(key, {}).setdefault(name, {})[v] = med
    for key, rows in table.items():
        print(f"\n{key} {a.dtype}: median ms over {a.rounds} process rounds ({a.knob})")
        for name, by in rows.items():
            print(f"  {name:28s} " + "  ".join(f"{v}: {by[v]:.4f}" for v in vals if v in by))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({k: v for k, v in table.items()}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
