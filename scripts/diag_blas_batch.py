"""Diag: hipBLASLt strided-batch GEMM (gemm_mode=blas) at the bench's pipeline-stage shapes.

Runs each (d, s) stage shape of the m=65536 n=k=1024 flagship once, validates against an fp32
reference, prints one line per case (flushes so a fault names its case)."""
import sys

import torch

sys.path.insert(0, ".")
from ddlb_amd.ops.gemm import gemm  # noqa: E402

m, n, k = 65536, 1024, 1024
g = torch.Generator(device="cuda").manual_seed(0)
A = (torch.rand((m, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
W = (torch.rand((n, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
ref = A.float() @ W.float().T
for d, s in [(2, 4), (4, 4), (8, 4), (8, 8), (2, 1)]:
    ml, rows = m // d, m // d // s
    C = torch.zeros((m, n), dtype=torch.bfloat16, device="cuda")
    for j in range(s):
        print(f"d={d} s={s} stage {j}: batch={d} rows={rows} gstride={ml}", flush=True)
        gemm(A[j * rows:], W, C[j * rows:], M=d * rows, a_grp=rows, a_gstride=ml, c_grp=rows,
             c_gstride=ml, mode="blas")
        torch.cuda.synchronize()
    err = (C.float() - ref).abs().max().item()
    print(f"d={d} s={s}: max|err| {err:.4f} {'ok' if err < 1e-3 * k else 'FAIL'}", flush=True)
