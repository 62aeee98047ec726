"""Why do side-stream ops of a plan sometimes take ~55 us each while a GEMM runs on stream 0?

The one-GPU budget (profiles/r04/r4_3_*) showed the RCCL-fed fused coll_pipeline emulation at
0.19 ms in one bind and 0.5-0.7 ms in others, every op of the comm stream (a copy kernel, a 1-block
signal kernel, even an event record) then taking ~55 us. This binds the SAME emulated plan several
times (each bind creates a new executor, i.e. new HIP streams) under variants, and prints the plan
time per bind and the mean side-stream op duration:

* ``base``       the plan as built (comm streams high priority, GEMM on the caller's stream);
* ``prio0``      every stream at normal priority;
* ``private``    the caller's stream is a fresh non-blocking torch stream, not the null stream;
* ``prio0+private``.

    python research/diag/diag_side_stream_stall.py [--candidate coll_pipeline/rccl/s8/fused] [--binds 4]
Run it again with GPU_MAX_HW_QUEUES=8 to vary the stream -> hardware-queue mapping.
"""

from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--candidate", default="coll_pipeline/rccl/s8/fused")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--binds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="base,prio0,private,prio0+private")
    a = ap.parse_args()

    import torch

    from plan_budget import candidate_cfgs
    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.algorithms import build_tp_columnwise
    from ddlb_amd.parallel.budget import PRESET, emulate, flag_buffers
    from ddlb_amd.parallel.plan import DT_BF16

    os.environ.setdefault("DDLB_CHILD_INIT_METHOD", "tcp://127.0.0.1:29519")
    comm = Communicator()
    comm.ensure_process_group()
    ctx = comm.native()
    cfg = [c for lbl, _, c in candidate_cfgs("tp_columnwise", "bfloat16", a.world)
           if lbl == a.candidate][0]
    plan, io = build_tp_columnwise(0, a.world, 65536, 1024, 1024, DT_BF16, DT_BF16, cfg)
    print(f"{a.candidate} world {a.world}  GPU_MAX_HW_QUEUES="
          f"{os.environ.get('GPU_MAX_HW_QUEUES', 'unset')}", flush=True)
    for var in a.variants.split(","):
        ep = emulate(plan)
        if "prio0" in var:
            ep.stream_priority = [0] * ep.nstreams
        stream = torch.cuda.Stream() if "private" in var else None
        times, side = [], []
        for _ in range(a.binds):
            bound = ctx.bind(ep)
            for name in flag_buffers(ep):
                bound.buffer(name).view(torch.int32).fill_(PRESET)
            torch.cuda.synchronize()
            with torch.cuda.stream(stream) if stream is not None else _null():
                for _ in range(5):
                    bound.run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    bound.run()
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / a.iters * 1e3)
                bound.set_timeline(True)
                bound.run()
                torch.cuda.synchronize()
                rows = bound.timeline()
                bound.set_timeline(False)
            side.append(statistics.mean(r["end_ms"] - r["start_ms"] for r in rows
                                        if r["stream"] != 0) * 1e3)
            bound.check_health()
            bound.close()
        print(f"  {var:16s} plan us per bind: {' '.join(f'{t:7.1f}' for t in times)}   "
              f"mean side-stream op us: {' '.join(f'{t:6.1f}' for t in side)}", flush=True)
    ctx.close()
    comm.destroy()
    return 0


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


if __name__ == "__main__":
    sys.exit(main())
