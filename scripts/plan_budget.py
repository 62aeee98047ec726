"""Per-rank budget of every N>1 bench candidate, emulated on ONE GPU (ddlb_amd.parallel.budget).

For each native candidate of ``bench.py``'s pool at ``--world`` ranks, rank ``--rank``'s plan is
built exactly as the job would build it, rewritten to its one-rank form (transfers -> local copies
of the same bytes on the same streams / engines, flags pre-set) and timed:

* ``gemm_ms``      its GEMMs alone, serialized, ungated (the compute floor of the schedule);
* ``plan_ms``      the whole emulated plan (GEMMs + concurrent copies + signal / wait ops), eager;
* ``graph_ms``     the same with hipGraph replay, where the plan is capturable;
* ``host_us``      host time of one ``run()`` call (enqueue only; the device is idle before it);
* op counts and the bytes the copies move;
* ``link_us``      a MODEL, not a measurement: the most loaded peer link's bytes
                   (``budget.link_bytes``) at ``--link-gbps`` per direction, i.e. the transfer
                   floor a real d-rank node adds beside the GEMM work.

EMULATED: local HBM copies stand in for xGMI links and no peer is ever late, so this is a budget
(a lower bound on rank 0's time), never a scaling value.

    python scripts/plan_budget.py --world 8 [--primitive tp_columnwise] [-m 65536 -n 1024 -k 1024]
           [--dtype bfloat16] [--candidates a,b] [--iters 20] [--out gpurun_out/budget.json]
           [--timeline a,b] [--rccl-blocks 6] [--variants "sig_side=1;gemm_first=0,s=8"]

``--rccl-blocks``: CU budget of the copy kernels standing in for RCCL (6 makes the stand-in
collectives link-slow, 32 HBM-fast); ``--variants``: ';'-separated AlgoConfig overrides, each
measured as an extra row ``<candidate>[<overrides>]`` beside the candidate itself.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def candidate_cfgs(primitive: str, dtype: str, world: int):
    """(label, options, AlgoConfig) of every native candidate bench.py can pick at ``world``."""
    import bench
    from ddlb_amd.primitives.native_common import algo_config
    from ddlb_amd.primitives.registry import resolve

    out = []
    for label, impl, opts in bench.candidate_pool(primitive, dtype, world):
        if impl != "native":
            continue
        opts = {k: v for k, v in opts.items() if not k.startswith("_")}
        cls, o, _ = resolve(primitive, impl, dict(opts))
        merged = {**cls.DEFAULT_OPTIONS, **o}
        for key, alias in cls.OPTION_ALIASES.items():
            merged[key] = alias.get(merged[key], merged[key])
        out.append((label, merged, algo_config(merged, order=merged.get("order", "AG_before"))))
    return out


def _time(bound, iters: int, warm: int = 5):
    import torch

    for _ in range(warm):
        bound.run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        bound.run()
    e1.record()
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / iters
    host = []
    for _ in range(max(iters // 2, 3)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bound.run()
        host.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    bound.check_health()
    return gpu_ms, sorted(host)[len(host) // 2]


def measure(ctx, plan, io, cfg_graph, iters: int, rccl_blocks: int, timeline: bool = False):
    import torch

    from ddlb_amd.parallel.budget import PRESET, emulate, flag_buffers, gemm_only
    from ddlb_amd.primitives.native_common import maybe_enable_graph

    ep = emulate(plan, rccl_blocks=rccl_blocks)
    res = {}
    for kind, p in (("plan", ep), ("gemm", gemm_only(ep))):
        bound = ctx.bind(p)
        try:
            for name in flag_buffers(p):
                bound.buffer(name).view(torch.int32).fill_(PRESET)
            for loc in (io.a, io.b):  # operands: U[-1, 1) (values do not change MFMA time)
                v = bound.view(loc)
                v.copy_((torch.rand(v.shape, device=v.device) * 2 - 1).to(v.dtype))
            torch.cuda.synchronize()
            res[f"{kind}_ms"], res[f"{kind}_host_us"] = _time(bound, iters)
            if kind == "plan" and timeline:
                from ddlb_amd.parallel.explain import format_timeline

                bound.set_timeline(True)
                for _ in range(3):
                    bound.run()
                torch.cuda.synchronize()
                res["timeline"] = format_timeline(bound.timeline())
                bound.set_timeline(False)
            if kind == "plan" and cfg_graph in (True, "auto"):
                try:
                    if maybe_enable_graph(bound, cfg_graph):
                        res["graph_ms"], res["graph_host_us"] = _time(bound, iters)
                except RuntimeError as e:
                    res["graph"] = f"not captured: {str(e)[:80]}"
        finally:
            bound.close()
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--primitive", default="tp_columnwise")
    ap.add_argument("-m", type=int, default=65536)
    ap.add_argument("-n", type=int, default=1024)
    ap.add_argument("-k", type=int, default=1024)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--candidates", default="")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rccl-blocks", type=int, default=32)
    ap.add_argument("--link-gbps", type=float, default=64.0,
                    help="per-direction xGMI link bandwidth of the link_us model (GB/s)")
    ap.add_argument("--out", default="")
    ap.add_argument("--timeline", default="",
                    help="comma list of candidates whose last eager run is printed as a per-op "
                         "timeline (ddlb_amd.parallel.explain.format_timeline)")
    ap.add_argument("--variants", default="",
                    help="';'-separated AlgoConfig overrides measured per candidate beside the "
                         "candidate itself, e.g. 'gemm_first=0;sig_side=0,gemm_first=0'")
    a = ap.parse_args(argv)

    import dataclasses

    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.algorithms import build_tp_columnwise, build_tp_rowwise
    from ddlb_amd.parallel.budget import copy_bytes, link_bytes, op_counts, signal_ops
    from ddlb_amd.primitives.native_common import dtype_codes

    os.environ.setdefault("DDLB_CHILD_INIT_METHOD", "tcp://127.0.0.1:29517")
    comm = Communicator()
    comm.ensure_process_group()
    ctx = comm.native()
    din, dout = dtype_codes(a.dtype)
    build = build_tp_columnwise if a.primitive == "tp_columnwise" else build_tp_rowwise
    want = [c.strip() for c in a.candidates.split(",") if c.strip()]
    rows = []
    print(f"EMULATED per-rank budget: rank {a.rank} of a {a.world}-rank {a.primitive} job, "
          f"m={a.m} n={a.n} k={a.k} {a.dtype} (local copies stand in for xGMI; not a scaling "
          f"value)", flush=True)
    print(f"{'candidate':44s} {'gemm_ms':>8s} {'plan_ms':>8s} {'graph_ms':>8s} {'host_us':>8s} "
          f"{'ops':>5s} {'sig':>4s} {'copyMB':>7s} {'link_us':>8s}", flush=True)
    todo = []
    for label, opts, cfg in candidate_cfgs(a.primitive, a.dtype, a.world):
        if want and label not in want:
            continue
        todo.append((label, opts, cfg))
        for var in [v.strip() for v in a.variants.split(";") if v.strip()]:
            kw = {}
            for item in var.split(","):
                key, val = item.split("=")
                cur = getattr(cfg, key.strip())
                kw[key.strip()] = (type(cur)(int(val)) if isinstance(cur, (bool, int))
                                   else type(cur)(val))
            todo.append((f"{label}[{var}]", opts, dataclasses.replace(cfg, **kw)))
    for label, opts, cfg in todo:
        row = {"candidate": label}
        try:
            plan, io = build(a.rank, a.world, a.m, a.n, a.k, din, dout, cfg)
            row.update(ops=len(plan.ops), signal_ops=signal_ops(plan),
                       counts=op_counts(plan))
            lb = link_bytes(plan)
            row["link_us"] = round(max(lb.values(), default=0) / (a.link_gbps * 1e3), 1)
            from ddlb_amd.parallel.budget import emulate
            row["copy_mb"] = round(copy_bytes(emulate(plan, a.rccl_blocks)) / 2 ** 20, 1)
            tl = [c.strip() for c in a.timeline.split(",") if c.strip()]
            row.update(measure(ctx, plan, io, opts.get("graph", "auto"), a.iters, a.rccl_blocks,
                               timeline=label in tl))
        except Exception as e:  # recorded, the sweep goes on
            row["error"] = f"{type(e).__name__}: {str(e)[:200]}"
        rows.append(row)

        def f(key, w=8):
            v = row.get(key)
            return f"{v:{w}.4f}" if isinstance(v, float) else f"{'-':>{w}s}"

        print(f"{label:44s} {f('gemm_ms')} {f('plan_ms')} {f('graph_ms')} "
              f"{row.get('plan_host_us', 0.0):8.1f} {row.get('ops', 0):5d} "
              f"{row.get('signal_ops', 0):4d} {row.get('copy_mb', 0.0):7.1f} "
              f"{row.get('link_us', 0.0):8.1f}"
              + (f"  {row['error']}" if "error" in row else ""), flush=True)
        if "timeline" in row:
            print(row["timeline"], flush=True)
        torch.cuda.synchronize()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump({"emulated": True, "world": a.world, "rank": a.rank,
                       "primitive": a.primitive, "m": a.m, "n": a.n, "k": a.k,
                       "dtype": a.dtype, "rows": rows}, fh, indent=1)
    ctx.close()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
