"""hipBLASLt algorithm autotune (csrc/gemm/blaslt.cpp) vs the heuristic's top-1 and torch's
F.linear, plus our MFMA kernel, on the flagship and per-shard shapes. Run twice:
DDLB_BLAS_TUNE=0 (top-1) and =1 (timed top-16); F.linear is the in-process constant."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddlb_amd.ops.gemm import gemm  # noqa: E402

SHAPES = [(65536, 1024, 1024), (8192, 1024, 1024), (16384, 1024, 1024), (8192, 1024, 8192),
          (65536, 1024, 8192), (16384, 8192, 1024), (8192, 8192, 8192), (4096, 4096, 4096)]


def timeit(fn, reps=50, rounds=5):
    out = []
    for _ in range(rounds):
        for _ in range(5):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps)
    return statistics.median(out) * 1e3


def main():
    tag = "tuned" if os.environ.get("DDLB_BLAS_TUNE", "1") != "0" else "top1"
    # pre-warm the clock
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(200):
        x @ x
    torch.cuda.synchronize()
    for m, n, k in SHAPES:
        A = (torch.rand((m, k), device="cuda") * 2 - 1).bfloat16()
        W = (torch.rand((n, k), device="cuda") * 2 - 1).bfloat16()
        C = torch.empty((m, n), device="cuda", dtype=torch.bfloat16)
        ref = A.float() @ W.float().T
        gemm(A, W, C, mode="blas")
        torch.cuda.synchronize()
        err = (C.float() - ref).abs().max().item()
        t_blas = timeit(lambda: gemm(A, W, C, mode="blas"))
        t_lin = timeit(lambda: torch.nn.functional.linear(A, W))
        t_own = timeit(lambda: gemm(A, W, C))
        tiles = {t: timeit(lambda: gemm(A, W, C, tile=t)) for t in ("t8", "pt8", "t4", "pt4")}
        tf = 2 * m * n * k / 1e12
        print(f"{m}x{n}x{k}: blas[{tag}] {t_blas:7.1f} us ({tf / t_blas * 1e6:6.0f} TF, err "
              f"{err:.3f})  F.linear {t_lin:7.1f} us  own {t_own:7.1f} us  " +
              "  ".join(f"{t} {v:7.1f}" for t, v in tiles.items()), flush=True)
        del A, W, C, ref


if __name__ == "__main__":
    main()
