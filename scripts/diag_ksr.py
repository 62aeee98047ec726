"""Diagnose the in-launch K-split reduction (GemmArgs::ks_ws) on one shape: where do wrong
outputs land (tile, 16-row x 32-col block), on which launch, and with which workspace fill.

    python scripts/diag_ksr.py [--shape 1024,512,4096] [--S 2]
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
    p.add_argument("--shape", default="1024,512,4096")
    p.add_argument("--S", type=int, default=2)
    a = p.parse_args()
    M, N, K = (int(x) for x in a.shape.split(","))
    S = a.S
    comm = Communicator()
    comm.ensure_process_group()
    tiles = (M // 256) * (N // 256)
    plan = Plan(0, 1, nstreams=1)
    A_ = plan.buffer("a", M * K * 2)
    B_ = plan.buffer("b", N * K * 2)
    C_ = plan.buffer("c", M * N * 2)
    ws = plan.buffer("ws", S * M * N * 4)
    cnt = plan.buffer("cnt", max(256, 8 * tiles), zero=True)
    plan.gemm(0, A_, B_, C_, M=M, N=N, K=K // S, lda=K, ldb=K, ldc=N, din=DT_BF16, dout=DT_BF16,
              tile=19, ksplit=S, ks_ws=ws, ks_cnt=cnt)
    ctx = NativeContext(comm)
    bound = ctx.bind(plan)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    bound.buffer("a").view(torch.bfloat16).view(M, K).copy_(A)
    bound.buffer("b").view(torch.bfloat16).view(N, K).copy_(W)
    ref = A.float() @ W.float().T
    parts = [(A[:, j * K // S:(j + 1) * K // S].float() @ W[:, j * K // S:(j + 1) * K // S].float().T)
             for j in range(S)]
    out = bound.buffer("c").view(torch.bfloat16).view(M, N)
    wsv = bound.buffer("ws").view(torch.float32)[:S * M * N].view(S, M, N)
    res = []
    for label, fill in [("nan-ws", float("nan")), ("nan-ws", float("nan")), ("zero-ws", 0.0),
                        ("keep-ws", None), ("keep-ws", None)]:
        out.fill_(float("nan"))
        if fill is not None:
            wsv.fill_(fill)
        torch.cuda.synchronize()
        bound.run()
        torch.cuda.synchronize()
        o = out.float()
        bad = ~((o - ref).abs() <= 2.0 ** -7 * ref.abs().max() + K * 2.0 ** -12)
        blocks = bad.view(M // 16, 16, N // 32, 32).any(3).any(1)
        nbad = int(blocks.sum())
        # which slab did the workspace receive (per tile: is slice j's partial present?)
        present = []
        for j in range(S):
            okj = ((wsv[j] - parts[j]).abs() <= 1e-2 * parts[j].abs().max()).view(
                M // 256, 256, N // 256, 256).all(3).all(1)
            present.append(int(okj.sum()))
        rows = sorted(set(int(r) for r in blocks.nonzero()[:, 0].tolist()))[:12]
        cols = sorted(set(int(c) for c in blocks.nonzero()[:, 1].tolist()))[:12]
        res.append({"run": label, "bad_16x32_blocks": nbad, "of": blocks.numel(),
                    "bad_row_blocks": rows, "bad_col_blocks": cols,
                    "nan_out": int(torch.isnan(o).sum()),
                    "ws_slices_present_per_tile": present,
                    "timeout": int(bound.ex.read_timeout())})
        print(json.dumps(res[-1]), flush=True)
    cv = bound.buffer("cnt").view(torch.int32)[:2 * tiles].view(tiles, 2).cpu().tolist()
    print(json.dumps({"counters": cv}), flush=True)
    bound.close()
    ctx.close()


if __name__ == "__main__":
    main()
