"""In-launch K-split reduction: does the memory type of the tile counters matter?

Runs the config #2 GEMM (8192 x 1024 x 8192, S = 2, ONE pt4 launch that reduces its slices
itself) as a plan, ``--runs`` times per variant, the f32 workspace refilled before every launch
(``--fill`` nan: a partial read before it landed is NaN; zero: it is a missing partial), and
counts the launches whose output misses the tight bound. Variants: the counters in uncached
(fine-grained) memory -- the binder's place for zero=True flag words -- or in ordinary cached
device memory like the workspace (what ``algorithms._full_gemm`` uses since r5_17).

    python scripts/diag_ksr_memtype.py --runs 30
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext
    from ddlb_amd.parallel.plan import DT_BF16, Plan

    p = argparse.ArgumentParser()
    p.add_argument("--runs", type=int, default=30)
    p.add_argument("--fill", default="nan", choices=["nan", "zero"])
    p.add_argument("-m", type=int, default=8192)
    p.add_argument("-n", type=int, default=1024)
    p.add_argument("-k", type=int, default=8192)
    p.add_argument("-S", type=int, default=2)
    a = p.parse_args()
    comm = Communicator()
    comm.ensure_process_group()
    M, N, K, S = a.m, a.n, a.k, a.S
    tiles = (M // 256) * (N // 256)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    ref = A.float() @ W.float().T
    bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
    ctx = NativeContext(comm)
    for uncached in (True, False):
        plan = Plan(0, 1, nstreams=1, stream_priority=[0])
        ra = plan.buffer("a", M * K * 2)
        rb = plan.buffer("b", N * K * 2)
        rc = plan.buffer("c", M * N * 2)
        ws = plan.buffer("ws", S * M * N * 4)
        cnt = plan.buffer("cnt", max(256, 8 * tiles), zero=uncached)
        plan.gemm(0, ra, rb, rc, M=M, N=N, K=K // S, lda=K, ldb=K, ldc=N, din=DT_BF16,
                  dout=DT_BF16, tile=19, ksplit=S, ks_ws=ws, ks_cnt=cnt)
        bound_plan = ctx.bind(plan)
        bound_plan.buffer("a").view(torch.bfloat16).view(M, K).copy_(A)
        bound_plan.buffer("b").view(torch.bfloat16).view(N, K).copy_(W)
        out = bound_plan.buffer("c").view(torch.bfloat16).view(M, N)
        wsv = bound_plan.buffer("ws").view(torch.float32)
        bad, worst, nelem = 0, 0.0, 0
        for _ in range(a.runs):
            wsv.fill_(float("nan") if a.fill == "nan" else 0.0)
            out.fill_(0)
            torch.cuda.synchronize()
            bound_plan.run()
            torch.cuda.synchronize()
            d = (out.float() - ref).abs()
            d = torch.nan_to_num(d, nan=float("inf"))
            e = float(d.max())
            if e > bound:
                bad += 1
                nelem += int((d > bound).sum())
            worst = max(worst, e)
        code = int(bound_plan.ex.read_timeout())
        bound_plan.close()
        print(json.dumps({"counters": "uncached" if uncached else "cached", "fill": a.fill,
                          "runs": a.runs, "bad_runs": bad, "bad_elements": nelem,
                          "worst_err": worst, "bound": bound, "timeout": code}), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
