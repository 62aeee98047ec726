"""Print (and optionally simulate) the native plan of a primitive/algorithm for one rank.

    python -m ddlb_amd.parallel.explain --primitive tp_columnwise -d 8 -m 65536 -n 1024 \
        -k 1024 --algorithm p2p_pipeline --backend ipc --rank 0
    python -m ddlb_amd.parallel.explain ... --simulate   # CPU run of all d ranks (small shapes)
    torchrun --nproc-per-node 8 -m ddlb_amd.parallel.explain -d 8 -m 65536 -n 1024 -k 1024 \
        --algorithm coll_pipeline --backend ipc -s 8 --timeline   # per-op GPU timeline per rank

The simulation executes every rank's plan on the CPU with the race / deadlock checker
(:mod:`ddlb_amd.parallel.sim`) — the same check the test-suite runs for every algorithm.
"""

from __future__ import annotations

import argparse

from typing import Dict, List

from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise, build_tp_rowwise
from ddlb_amd.parallel.plan import NAME_DT, SIG_KERNEL, SIG_STREAM

# one letter per op kind in the timeline bars
_GLYPH = {"gemm": "G", "allgather": "A", "reduce_scatter": "R", "send": "S", "recv": "V",
          "copy": "c", "copy_multi": "c", "reduce": "+", "signal": "!", "wait_signal": "w",
          "wait": ".", "record": "|", "memset": "0", "group_start": "(", "group_end": ")"}


def format_timeline(rows: List[Dict], width: int = 72) -> str:
    """Text Gantt of :meth:`BoundPlan.timeline` rows: one bar per stream (letters = op kinds,
    ``.`` = blocked on a dependency), then the ops sorted by start and a busy / overlap summary
    (busy = time in GEMM / comm / copy / reduce ops, not in waits)."""
    if not rows:
        return "(empty plan)"
    span = max(r["end_ms"] for r in rows) or 1e-9
    streams = sorted({r["stream"] for r in rows})
    lines = [f"timeline: {span * 1e3:.1f} us from fork to the last op, {len(rows)} ops"]
    busy_kinds = {"gemm", "allgather", "reduce_scatter", "send", "recv", "copy", "copy_multi",
                  "reduce", "memset"}
    busy_total = 0.0
    for st in streams:
        bar = [" "] * width
        busy = 0.0
        for r in rows:
            if r["stream"] != st:
                continue
            a = int(r["start_ms"] / span * (width - 1))
            b = max(a, int(r["end_ms"] / span * (width - 1)))
            ch = _GLYPH.get(r["op"], "?")
            for x in range(a, b + 1):
                if bar[x] in (" ", ".", "|") or ch not in (".", "|"):
                    bar[x] = ch
            if r["op"] in busy_kinds:
                busy += r["end_ms"] - r["start_ms"]
        busy_total += busy
        lines.append(f"  s{st:<2d} |{''.join(bar)}| busy {busy * 1e3:8.1f} us")
    lines.append(f"  sum of busy time over streams / span = {busy_total / span:.2f} "
                 "(> 1: streams overlap)")
    if any("host_us" in r for r in rows):
        per_kind: Dict[str, float] = {}
        for r in rows:
            per_kind[r["op"]] = per_kind.get(r["op"], 0.0) + r.get("host_us", 0.0)
        total = sum(per_kind.values())
        top = ", ".join(f"{k} {v:.0f}" for k, v in sorted(per_kind.items(), key=lambda x: -x[1])[:6])
        lines.append(f"  host enqueue {total:.0f} us: {top}")
    lines.append("  idx stream op               start_us    end_us   dur_us")
    for r in sorted(rows, key=lambda r: (r["start_ms"], r["index"])):
        if r["end_ms"] - r["start_ms"] < 1e-6 and r["op"] in ("record", "group_start"):
            continue
        lines.append(f"  {r['index']:3d} s{r['stream']:<5d} {r['op']:14s} "
                     f"{r['start_ms'] * 1e3:9.1f} {r['end_ms'] * 1e3:9.1f} "
                     f"{(r['end_ms'] - r['start_ms']) * 1e3:8.1f}")
    return "\n".join(lines)


def gpu_timeline(a) -> None:
    """Build the native implementation for this rank (launched under torchrun for d > 1), warm
    it up, run once with per-op timing events and print this rank's timeline."""
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.primitives.registry import resolve

    comm = Communicator()
    comm.ensure_process_group()
    opts = {"algorithm": a.algorithm, "backend": a.backend, "s": a.s,
            "multicast_protocol": a.protocol, "signal": a.signal,
            "offset_stream_indexing_by_rank": not a.no_ring, "fused": a.fused}
    if a.primitive == "tp_columnwise":
        opts["order"] = a.order
    if a.graph:
        opts["graph"] = True
    cls, opts, _ = resolve(a.primitive, "native", opts)
    impl = cls(m=a.m, n=a.n, k=a.k, dtype=a.dtype, **opts)
    for _ in range(5):
        impl.run()
    torch.cuda.synchronize()
    comm.barrier()
    # host cost of enqueueing one run (every HIP / RCCL call of the plan), GPU kept busy
    import time

    host = []
    for _ in range(20):
        t0 = time.perf_counter()
        impl.run()
        host.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    comm.barrier()
    host.sort()
    if a.graph:  # one hipGraphLaunch per run: no per-op timeline inside a replayed graph
        out = impl.run()
        torch.cuda.synchronize()
        impl.validate(out)
        if comm.rank == 0:
            print(f"[rank 0/{comm.world_size}] {a.primitive} {a.algorithm}/{a.backend} graph "
                  f"replay: {len(impl.plan.ops)} plan ops, host enqueue per run "
                  f"{host[len(host) // 2]:.0f} us (median of 20)", flush=True)
        impl.close()
        comm.destroy()
        return
    impl.bound.set_timeline(True)
    out = impl.run()
    torch.cuda.synchronize()
    rows = impl.bound.timeline()
    impl.validate(out)
    text = format_timeline(rows)
    for r in range(comm.world_size):
        if r == comm.rank:
            print(f"[rank {comm.rank}/{comm.world_size}] {a.primitive} {a.algorithm}/{a.backend} "
                  f"m={a.m} n={a.n} k={a.k} {a.dtype}: {len(impl.plan.ops)} plan ops, host "
                  f"enqueue per run {host[len(host) // 2]:.0f} us (median of 20)\n{text}",
                  flush=True)
        comm.barrier()
    impl.bound.set_timeline(False)
    impl.close()
    comm.destroy()


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--primitive", default="tp_columnwise", choices=["tp_columnwise", "tp_rowwise"])
    p.add_argument("-d", "--world", type=int, default=2)
    p.add_argument("--rank", type=int, default=0)
    p.add_argument("-m", type=int, default=64)
    p.add_argument("-n", type=int, default=16)
    p.add_argument("-k", type=int, default=32)
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--algorithm", default="default")
    p.add_argument("--backend", default="rccl")
    p.add_argument("--order", default="AG_before")
    p.add_argument("-s", type=int, default=2)
    p.add_argument("--protocol", default="memcpy")
    p.add_argument("--signal", "--signal-method", dest="signal", default="stream",
                   choices=["stream", "kernel"])  # (torchrun's parser claims "--signal...")
    p.add_argument("--no-ring", action="store_true")
    p.add_argument("--fused", action="store_true")
    p.add_argument("--simulate", action="store_true")
    p.add_argument("--graph", action="store_true",
                   help="with --timeline: capture the plan in a hipGraph and report the host "
                        "cost of a replayed run instead of the per-op timeline")
    p.add_argument("--timeline", action="store_true",
                   help="run the plan on the GPU (world from the launcher's env, not -d) and "
                        "print its per-op timeline")
    a = p.parse_args(argv)
    if a.timeline:
        gpu_timeline(a)
        return
    cfg = AlgoConfig(algorithm=a.algorithm, backend=a.backend, order=a.order, s=a.s,
                     ring=not a.no_ring, protocol=a.protocol,
                     signal=SIG_STREAM if a.signal == "stream" else SIG_KERNEL, fused=a.fused)
    din = NAME_DT[a.dtype]
    dout = NAME_DT["bfloat16"] if a.dtype == "float8_e4m3fn" else din
    build = build_tp_columnwise if a.primitive == "tp_columnwise" else build_tp_rowwise
    plan, io = build(a.rank, a.world, a.m, a.n, a.k, din, dout, cfg)
    print(plan.describe())
    print(f"  inputs: A={io.a}  B={io.b}\n  output: {io.out}")
    if a.simulate:
        import torch

        from ddlb_amd.parallel.sim import Simulator, make_buffers, read_tensor, write_tensor

        built = [build(r, a.world, a.m, a.n, a.k, din, dout, cfg) for r in range(a.world)]
        bufs = make_buffers([b[0] for b in built])
        g = torch.Generator().manual_seed(0)
        A = torch.randint(-2, 3, (a.m, a.k), generator=g).float()
        B = torch.randint(-2, 3, (a.k, a.n), generator=g).float()
        tdt = read_tensor(bufs[0], built[0][1].a).dtype
        for r, (_, rio) in enumerate(built):
            if a.primitive == "tp_columnwise":
                ml = a.m // a.world
                write_tensor(bufs[r], rio.a, A[r * ml:(r + 1) * ml].to(tdt))
                write_tensor(bufs[r], rio.b, B.t().contiguous().to(tdt))
            else:
                kl = a.k // a.world
                write_tensor(bufs[r], rio.a, A[:, r * kl:(r + 1) * kl].contiguous().to(tdt))
                write_tensor(bufs[r], rio.b, B[r * kl:(r + 1) * kl].t().contiguous().to(tdt))
        sim = Simulator([b[0] for b in built], bufs)
        for _ in range(3):
            sim.run_epoch()
        ref = A @ B
        worst = 0.0
        for r, (_, rio) in enumerate(built):
            out = read_tensor(bufs[r], rio.out).float()
            want = ref if a.primitive == "tp_columnwise" else ref[
                r * (a.m // a.world):(r + 1) * (a.m // a.world)]
            worst = max(worst, float((out - want).abs().max()))
        print(f"simulated {a.world} ranks x 3 epochs: no race, no deadlock, max|err| = {worst}")


if __name__ == "__main__":
    main()
