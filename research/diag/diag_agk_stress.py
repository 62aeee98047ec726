"""Stress of the in-kernel all-gather's publication (tests/test_native_gpu.py
test_in_kernel_allgather_world1, many more launches): the peer rows of the gather buffer are
NaN before every launch, the copy workgroups pull them, publish (AgMode variants) and the gated
tiles consume them; counts the launches whose C misses the fp32 reference. The in-launch K-split
showed that a fence-free publication can pass 10 launches and fail 1 in 10-30 (r5_18).

    python research/diag/diag_agk_stress.py --runs 100 --modes 0,6,14,30
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext
    from ddlb_amd.parallel.plan import DT_BF16, Plan, SIG_IN_LAUNCH, SIG_KERNEL, SIG_STREAM

    p = argparse.ArgumentParser()
    p.add_argument("--runs", type=int, default=100)
    p.add_argument("--modes", default="0,6,14,30")
    p.add_argument("--graph", type=int, default=1)
    a = p.parse_args()
    comm = Communicator()
    comm.ensure_process_group()
    M, N, K, nsub = 32768, 1024, 1024, 4
    half, rows = M // 2, M // (2 * nsub)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    ref = A.float() @ W.float().T
    ctx = NativeContext(comm)
    for mode in (int(x) for x in a.modes.split(",")):
        graph = bool(a.graph)
        plan = Plan(0, 1, nstreams=1, stream_priority=[0])
        ra = plan.buffer("a", M * K * 2)
        peer = plan.buffer("peer", M * K * 2)
        bt = plan.buffer("bt", N * K * 2)
        c = plan.buffer("c", M * N * 2)
        fl = plan.buffer("flags", 256, zero=True)
        READY, ACK, ARRIVE, CNT = fl, fl + 8, fl + 16, fl + 48
        sig = SIG_KERNEL if graph else SIG_STREAM
        plan.signal(0, [READY + 4], method=sig)
        plan.signal(0, [ARRIVE + 4 * j for j in range(nsub)], method=sig)
        ag = dict(ctas=32, parts=8, rank=0, src=[ra, peer], ack=[ACK, ACK + 4], ready=READY,
                  count=CNT, mode=mode, wait_acks=[ACK, ACK + 4] if mode & 16 else None)
        plan.gemm(0, ra, bt, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, din=DT_BF16, dout=DT_BF16,
                  tile=19, flags=ARRIVE, flag_rows=rows, nshards=2 * nsub, nsub=nsub,
                  first_shard=0, tile_order=1, ag=ag)
        plan.wait_signal(0, [ACK + 4], method=SIG_IN_LAUNCH if mode & 16 else sig)
        bound = ctx.bind(plan)
        if graph:
            bound.enable_graph(True)
        av = bound.buffer("a").view(torch.bfloat16).view(M, K)
        av[:half].copy_(A[:half])
        bound.buffer("peer").view(torch.bfloat16).view(M, K)[half:].copy_(A[half:])
        bound.buffer("bt").view(torch.bfloat16).view(N, K).copy_(W)
        out = bound.buffer("c").view(torch.bfloat16).view(M, N)
        bad, nel, worst = 0, 0, 0.0
        for _ in range(a.runs):
            av[half:].fill_(float("nan"))
            out.zero_()
            torch.cuda.synchronize()
            bound.run()
            torch.cuda.synchronize()
            d = torch.nan_to_num((out.float() - ref).abs(), nan=float("inf"))
            e = float(d.max())
            if e > 1e-3 * K:
                bad += 1
                nel += int((d > 1e-3 * K).sum())
            worst = max(worst, e)
        code = int(bound.ex.read_timeout())
        bound.close()
        print(json.dumps({"mode": mode, "graph": graph, "runs": a.runs, "bad_runs": bad,
                          "bad_elements": nel, "worst_err": worst, "timeout": code}), flush=True)
        if code:
            break
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
