"""Same hipBLASLt kernel, two callers: our plan's blas mode vs torch F.linear (flagship shape).
Run under rocprofv3 --kernel-trace to compare the dispatches (grid, workgroup, LDS, VGPRs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddlb_amd.ops.gemm import gemm  # noqa: E402

m, n, k = 65536, 1024, 1024
A = (torch.rand((m, k), device="cuda") * 2 - 1).bfloat16()
W = (torch.rand((n, k), device="cuda") * 2 - 1).bfloat16()
C = torch.empty((m, n), device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    gemm(A, W, C, mode="blas")
    torch.nn.functional.linear(A, W)
torch.cuda.synchronize()
for _ in range(20):
    gemm(A, W, C, mode="blas")
torch.cuda.synchronize()
for _ in range(20):
    torch.nn.functional.linear(A, W)
torch.cuda.synchronize()
print("done")
