"""fp8 e4m3 flagship-shape GEMM: plain fp8 MFMA vs block-scaled MX on each t-kernel, and
hipBLASLt _scaled_mm (unit scales) as the vendor reference."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddlb_amd.ops.gemm import gemm  # noqa: E402


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


x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(200):
    x @ x
for m, n, k in [(65536, 1024, 1024), (8192, 8192, 8192)]:
    A = (torch.rand((m, k), device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
    W = (torch.rand((n, k), device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
    C = torch.empty((m, n), device="cuda", dtype=torch.bfloat16)
    one = torch.ones((), device="cuda")
    res = {"_scaled_mm": timeit(lambda: torch._scaled_mm(A, W.t(), scale_a=one, scale_b=one,
                                                         out_dtype=torch.bfloat16))}
    for mode in ("auto", "mx"):
        for tile in ("auto", "t8", "pt8", "t4", "pt4"):
            res[f"{mode}/{tile}"] = timeit(lambda: gemm(A, W, C, mode=mode, tile=tile))
    tf = 2 * m * n * k / 1e12
    print(f"{m}x{n}x{k} fp8: " + "  ".join(f"{k_} {v:.1f}us({tf / v * 1e6:.0f}TF)"
                                          for k_, v in res.items()), flush=True)
