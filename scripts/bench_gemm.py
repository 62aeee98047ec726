"""Microbenchmark: native MFMA GEMM vs torch.matmul (hipBLASLt) on the shapes the primitives run.

Variants are interleaved in ONE process, several rounds, median reported (cdna guide §5.4 rule 24).
Random U[-1,1) operands (rule 25). Output: a table on stdout and JSON (``--json``).

    python scripts/bench_gemm.py --json gpurun_out/gemm.json
"""

from __future__ import annotations

import argparse
import json
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (M, N, K, note)
    (65536, 1024, 1024, "tp_col m=65536 full GEMM (bench.py config)"),
    (8192, 1024, 1024, "tp_col m=65536 d=8 per-shard GEMM"),
    (65536, 1024, 8192, "tp_col m=65536 k=8192"),
    (8192, 1024, 8192, "tp_col m=8192 n=1024 k=8192 (BASELINE #2 full GEMM)"),
    (16384, 8192, 1024, "tp_row m=16384 k=8192 d=8 local partial"),
    (16384, 8192, 8192, "tp_row m=16384 k=8192 d=1"),
    (8192, 8192, 8192, "square 8k"),
    (4096, 4096, 4096, "square 4k"),
]


def timeit(fn, iters, warm=3):
    import torch

    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    import torch

    from ddlb_amd.ops.gemm import gemm

    p = argparse.ArgumentParser()
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--tiles", default="auto,pt4,t4,256x256,128x128")
    p.add_argument("--modes", default="auto")
    p.add_argument("--shapes", default="all")
    p.add_argument("--json", default=None)
    p.add_argument("--check", action="store_true", help="tight numerics check first")
    a = p.parse_args()
    dt = getattr(torch, a.dtype)
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    shapes = SHAPES if a.shapes == "all" else [SHAPES[int(i)] for i in a.shapes.split(",")]
    results = []
    for (M, N, K, note) in shapes:
        A = (torch.rand((M, K), generator=g, device="cuda") * 2 - 1).to(dt)
        W = (torch.rand((N, K), generator=g, device="cuda") * 2 - 1).to(dt)
        odt = torch.bfloat16 if dt == torch.float8_e4m3fn else dt
        out = torch.empty((M, N), dtype=odt, device="cuda")
        Bkn = W.t().contiguous()
        variants = {}
        if dt == torch.float8_e4m3fn:
            one = torch.ones((), device="cuda")
            Bcol = W.t()  # [K,N] column-major view of the [N,K] row-major weight
            try:
                torch._scaled_mm(A, Bcol, scale_a=one, scale_b=one, out_dtype=odt)
                variants["hipblaslt_scaled_mm"] = lambda: torch._scaled_mm(
                    A, Bcol, scale_a=one, scale_b=one, out_dtype=odt)
            except Exception as e:
                print("scaled_mm unavailable:", e)
        else:
            variants["hipblaslt"] = lambda: torch.matmul(A, Bkn, out=out)
            # the K-contiguous weight layout (te.Linear / F.linear), hipBLASLt's fastest form
            variants["hipblaslt_linear"] = lambda: torch.nn.functional.linear(A, W)
        for t in a.tiles.split(","):
            for mode in a.modes.split(","):
                variants[f"native[{t},{mode}]"] = (lambda t=t, mode=mode: gemm(A, W, out, tile=t,
                                                                               mode=mode))
        if a.check:  # tight numerics of every native variant before timing it
            ref = A.float() @ W.float().t()
            bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
            for k, fn in variants.items():
                if not k.startswith("native"):
                    continue
                out.fill_(float("nan"))
                fn()
                torch.cuda.synchronize()
                err = float((out.float() - ref).abs().max())
                print(f"  check {k:24s} max|err| {err:.4g} (bound {bound:.4g}) "
                      f"{'ok' if err <= bound else 'FAIL'}")
            del ref
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(timeit(fn, a.iters))
        flop = 2.0 * M * N * K
        row = {"M": M, "N": N, "K": K, "dtype": a.dtype, "note": note, "variants": {}}
        print(f"\n{M}x{N}x{K} {a.dtype}  ({note})")
        for k, ts in times.items():
            med = statistics.median(ts)
            tf = flop / (med * 1e-3) / 1e12
            row["variants"][k] = {"ms_median": med, "ms_min": min(ts), "tflops": tf}
            print(f"  {k:28s} {med:8.4f} ms  {tf:8.1f} TFLOP/s")
        results.append(row)
        del A, W, out, Bkn
        torch.cuda.empty_cache()
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
