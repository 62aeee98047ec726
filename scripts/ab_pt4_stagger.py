"""A/B of the ungated pt4's start stagger (GemmArgs::stagger_ns, ``C.set_pt4_stagger_ns``): half
the CUs (every odd 8-workgroup group, one per XCD) sleep ``ns`` before their first tile, so the
two halves run out of phase and one half's C-store bursts and A loads overlap the other half's
MFMAs instead of every CU hitting HBM at the same time.

Variants are interleaved in ONE process over several rounds, median reported (cdna guide §5.4
rule 24); each variant is first checked against fp32 (tight bound) and repeat-identical 20x.

    python scripts/ab_pt4_stagger.py --ns 0,2000,4000,6000 [--rounds 7] [--iters 30]
"""

from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # (M, N, K, dtype, mode, label)
    (65536, 1024, 1024, "bfloat16", "auto", "flagship bf16"),
    (65536, 1024, 1024, "float8_e4m3fn", "mx", "flagship MX-fp8"),
    (16384, 8192, 1024, "bfloat16", "auto", "row partial 16384x8192x1024"),
    (8192, 8192, 8192, "bfloat16", "auto", "8192^3 bf16"),
]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="0,2000,4000,6000")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default="", help="comma list of shape indices (default: all)")
    a = ap.parse_args()

    import torch

    from ddlb_amd.ops import load
    from ddlb_amd.ops.gemm import gemm

    C = load()
    vals = [int(x) for x in a.ns.split(",")]
    g = torch.Generator(device="cuda").manual_seed(3)
    shapes = SHAPES if not a.shapes else [SHAPES[int(i)] for i in a.shapes.split(",")]
    for M, N, K, dt, mode, label in shapes:
        tdt = getattr(torch, dt)
        A = (torch.rand((M, K), generator=g, device="cuda") * 2 - 1).to(tdt)
        W = (torch.rand((N, K), generator=g, device="cuda") * 2 - 1).to(tdt)
        out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
        ref = A.float() @ W.float().t()
        bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
        ok = {}
        for v in vals:
            C.set_pt4_stagger_ns(v)
            gemm(A, W, out, tile="pt4", mode=mode)
            torch.cuda.synchronize()
            first = out.clone()
            err = float((first.float() - ref).abs().max())
            for _ in range(20):
                gemm(A, W, out, tile="pt4", mode=mode)
            torch.cuda.synchronize()
            same = torch.equal(out, first)
            ok[v] = err <= bound and same
            if not ok[v]:
                print(f"  {label}: stagger {v} FAILED (max|err| {err:.4g} bound {bound:.4g}, "
                      f"repeat-identical {same})", flush=True)
        del ref
        times = {v: [] for v in vals}
        for _ in range(a.rounds):
            for v in vals:
                C.set_pt4_stagger_ns(v)
                for _ in range(3):
                    gemm(A, W, out, tile="pt4", mode=mode)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    gemm(A, W, out, tile="pt4", mode=mode)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
        flop = 2.0 * M * N * K
        print(f"{label:30s} " + "  ".join(
            f"{v:5d} ns: {statistics.median(times[v]):7.2f} us "
            f"({flop / statistics.median(times[v]) / 1e6:5.0f} TF){'' if ok[v] else ' INVALID'}"
            for v in vals), flush=True)
    C.set_pt4_stagger_ns(0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
