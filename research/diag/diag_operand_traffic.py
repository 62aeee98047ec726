"""What the flagship GEMM's operand traffic costs: the same pt4 launch (65536 x 1024 x 1024 bf16
by default) with A's row pitch set to 0 (every A row is row 0: A comes from L2 / L1, no HBM
stream), with A's and B's pitches 0 (no operand traffic beyond one row each), and as is. C is
written in full in every form. Timing-only: the pitch-0 forms compute a different product.

    python research/diag/diag_operand_traffic.py --shapes 65536x1024x1024,65536x1024x8192
"""

from __future__ import annotations

import argparse
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ddlb_amd.ops import gemm as G

    p = argparse.ArgumentParser()
    p.add_argument("--shapes", default="65536x1024x1024,65536x1024x8192")
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()
    C = G.load()
    dt = getattr(torch, a.dtype)
    mode = "mx" if dt == torch.float8_e4m3fn else "auto"
    for shp in a.shapes.split(","):
        M, N, K = (int(x) for x in shp.split("x"))
        A = (torch.rand((M, K), device="cuda") * 2 - 1).to(dt)
        W = (torch.rand((N, K), device="cuda") * 2 - 1).to(dt)
        out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        din = G.dtype_code(dt)

        def launch(lda, ldb):
            C.gemm(A.data_ptr(), W.data_ptr(), out.data_ptr(), lda, ldb, N, M, N, K, din,
                   G.DT_BF16, G.TILES["pt4"], G.MODES[mode], 0, 0, 0, 0, s, 0, 1)

        forms = {"as is": (K, K), "A pitch 0": (0, K), "A and B pitch 0": (0, 0)}
        times = {k: [] for k in forms}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for k, (lda, ldb) in forms.items():
                for _ in range(3):
                    launch(lda, ldb)
                torch.cuda.synchronize()
                ev0.record()
                for _ in range(a.iters):
                    launch(lda, ldb)
                ev1.record()
                torch.cuda.synchronize()
                times[k].append(ev0.elapsed_time(ev1) / a.iters)
        print(f"\n{M}x{N}x{K} {a.dtype} pt4: median ms over {a.rounds} rounds", flush=True)
        for k, ts in times.items():
            print(f"  {k:18s} {statistics.median(ts):.4f}", flush=True)
        del A, W, out
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
