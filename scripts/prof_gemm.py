"""Run one GEMM variant N times (for rocprofv3 --kernel-trace / --pmc profiles)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ddlb_amd.ops.gemm import gemm

    p = argparse.ArgumentParser()
    p.add_argument("-m", type=int, default=65536)
    p.add_argument("-n", type=int, default=1024)
    p.add_argument("-k", type=int, default=1024)
    p.add_argument("--tiles", default="256x256,pt4,128x128")
    p.add_argument("--hipblaslt", action="store_true",
                   help="also the vendor GEMM (F.linear: hipBLASLt, K-contiguous weight)")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float8_e4m3fn"])
    p.add_argument("--mode", default="auto", help="auto | mx (block-scaled fp8 MFMA)")
    a = p.parse_args()
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    dt = getattr(torch, a.dtype)
    A = (torch.rand((a.m, a.k), generator=g, device="cuda") * 2 - 1).to(dt)
    W = (torch.rand((a.n, a.k), generator=g, device="cuda") * 2 - 1).to(dt)
    out = torch.empty((a.m, a.n), dtype=torch.bfloat16, device="cuda")
    for t in [t for t in a.tiles.split(",") if t]:
        for _ in range(a.iters):
            gemm(A, W, out, tile=t, mode=a.mode)
    if a.hipblaslt:
        if dt == torch.float8_e4m3fn:  # the vendor fp8 GEMM: hipBLASLt through _scaled_mm
            one = torch.ones((), device="cuda")
            for _ in range(a.iters):
                torch._scaled_mm(A, W.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        else:
            for _ in range(a.iters):
                torch.nn.functional.linear(A, W)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
