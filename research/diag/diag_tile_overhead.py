"""Split the flagship pt4 GEMM's time into per-K-tile work and a fixed per-tile cost.

For N = 1024 and M in {65536, 131072} (4 and 8 tiles per workgroup on 256 CUs) and K over a
range, the median time (interleaved rounds, one process) is fitted with

    T(M, K) = L + R(M) * (nk(K) * k + o)       R = tiles / workgroups, nk = K-tiles per tile

by least squares: ``k`` = time per K-tile step, ``o`` = fixed cost per tile (C epilogue, tile
switch, pipeline refill), ``L`` = launch / fill / drain. bf16 and MX-fp8 (128-byte K-tiles: 64
bf16 or 128 fp8 elements).

    python research/diag/diag_tile_overhead.py [--rounds 5] [--iters 20]
"""

from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()

    import numpy as np
    import torch

    from ddlb_amd.ops import load
    from ddlb_amd.ops.gemm import gemm

    C = load()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    N = 1024
    cases = {"bf16": (torch.bfloat16, "auto", [512, 1024, 2048, 4096]),
             "mx-fp8": (torch.float8_e4m3fn, "mx", [1024, 2048, 4096, 8192])}
    for name, (tdt, mode, ks) in cases.items():
        esz = torch.tensor([], dtype=tdt).element_size()
        runs = []
        for M in (65536, 131072):
            for K in ks:
                A = (torch.rand((M, K), device="cuda") * 2 - 1).to(tdt)
                W = (torch.rand((N, K), device="cuda") * 2 - 1).to(tdt)
                out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
                runs.append((M, K, A, W, out))
        times = {(M, K): [] for M, K, *_ in runs}
        for _ in range(a.rounds):
            for M, K, A, W, out in runs:
                for _ in range(3):
                    gemm(A, W, out, tile="pt4", mode=mode)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    gemm(A, W, out, tile="pt4", mode=mode)
                e1.record()
                torch.cuda.synchronize()
                times[(M, K)].append(e0.elapsed_time(e1) / a.iters * 1e3)
        rows, ys = [], []
        for (M, K), ts in times.items():
            t = statistics.median(ts)
            R = (M // 256) * (N // 256) / ncu
            nk = K * esz // 128
            rows.append([1.0, R * nk, R])
            ys.append(t)
            print(f"{name:7s} M={M:6d} K={K:5d} tiles/WG={R:4.1f} nk={nk:3d}  {t:8.2f} us  "
                  f"({2.0 * M * N * K / t / 1e6:5.0f} TF)", flush=True)
        (L, k, o), res, *_ = np.linalg.lstsq(np.array(rows), np.array(ys), rcond=None)
        fit = np.array(rows) @ np.array([L, k, o])
        worst = float(np.max(np.abs(fit - np.array(ys)) / np.array(ys)))
        print(f"{name:7s} fit: per K-tile step k = {k:.3f} us, per tile o = {o:.2f} us, "
              f"launch/fill L = {L:.2f} us (worst residual {worst * 100:.1f} %); flagship "
              f"(4 tiles/WG, nk = {1024 * esz // 128}): o share "
              f"{4 * o / (L + 4 * (1024 * esz // 128 * k + o)) * 100:.0f} %", flush=True)
        del runs
        torch.cuda.empty_cache()
    del C
    return 0


if __name__ == "__main__":
    sys.exit(main())
