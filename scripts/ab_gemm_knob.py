"""A/B of a GEMM kernel switch (GemmArgs::knob, ``C.set_gemm_knob``) on the primitives' shapes:
variants interleaved in ONE process, several rounds, median (cdna guide §5.4 rule 24); each
variant is first checked against fp32 (tight bound) and repeat-identical 20x.

    python scripts/ab_gemm_knob.py --knobs 0,1 [--rounds 7] [--iters 30]
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
    (8192, 8192, 8192, "float8_e4m3fn", "mx", "8192^3 MX-fp8"),
]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--knobs", default="0,1")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--tile", default="pt4")
    a = ap.parse_args()

    import torch

    from ddlb_amd.ops import load
    from ddlb_amd.ops.gemm import gemm

    C = load()
    knobs = [int(x) for x in a.knobs.split(",")]
    g = torch.Generator(device="cuda").manual_seed(3)
    for M, N, K, dt, mode, label in SHAPES:
        tdt = getattr(torch, dt)
        A = (torch.rand((M, K), generator=g, device="cuda") * 2 - 1).to(tdt)
        W = (torch.rand((N, K), generator=g, device="cuda") * 2 - 1).to(tdt)
        out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
        ref = A.float() @ W.float().t()
        bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
        ok = {}
        for kb in knobs:
            C.set_gemm_knob(kb)
            gemm(A, W, out, tile=a.tile, mode=mode)
            torch.cuda.synchronize()
            first = out.clone()
            err = float((first.float() - ref).abs().max())
            same = True
            for _ in range(20):
                gemm(A, W, out, tile=a.tile, mode=mode)
            torch.cuda.synchronize()
            same = torch.equal(out, first)
            ok[kb] = err <= bound and same
            if not ok[kb]:
                print(f"  {label}: knob {kb} FAILED (max|err| {err:.4g} bound {bound:.4g}, "
                      f"repeat-identical {same})", flush=True)
        del ref
        times = {kb: [] for kb in knobs}
        for _ in range(a.rounds):
            for kb in knobs:
                C.set_gemm_knob(kb)
                for _ in range(3):
                    gemm(A, W, out, tile=a.tile, mode=mode)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    gemm(A, W, out, tile=a.tile, mode=mode)
                e1.record()
                torch.cuda.synchronize()
                times[kb].append(e0.elapsed_time(e1) / a.iters * 1e3)
        flop = 2.0 * M * N * K
        print(f"{label:34s} " + "  ".join(
            f"knob {kb}: {statistics.median(times[kb]):8.2f} us "
            f"({flop / statistics.median(times[kb]) / 1e6:6.0f} TF){'' if ok[kb] else ' INVALID'}"
            for kb in knobs), flush=True)
    C.set_gemm_knob(0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
