"""A/B of the ways to run a few-tile, long-K GEMM (fewer 256x256 tiles than CUs), one process,
interleaved rounds, median (cdna guide §5.4 rule 24):

  unsplit[<tile>]      one launch of <tile> over the whole K
  ks<S>[pt4]/reduce    pt4 runs every (slice, tile) pair in one launch into output-dtype
                       partials, then the reduce kernel sums them (the plans' ``_full_gemm``)
  ks<S>[pt4]/reduce-f32  the same with f32 partials, rounded once by the reduce

    python research/diag/ab_ksplit_forms.py --dtype bfloat16 --shapes 8192x1024x8192,4096x1024x8192
"""

from __future__ import annotations

import argparse
import re
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ddlb_amd.ops import gemm as G

    p = argparse.ArgumentParser()
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--shapes", default="8192x1024x8192")
    p.add_argument("--tiles", default="pt4,256x128,128x256")
    p.add_argument("--splits", default="2,4")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--checks", type=int, default=3, help="checked calls per variant")
    p.add_argument("--only", default=None, help="regex: run the matching variants only")
    a = p.parse_args()
    C = G.load()
    dt = getattr(torch, a.dtype)
    mode = "mx" if dt == torch.float8_e4m3fn else "auto"
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    for shp in a.shapes.split(","):
        M, N, K = (int(x) for x in shp.split("x"))
        A = (torch.rand((M, K), generator=gen, device="cuda") * 2 - 1).to(dt)
        W = (torch.rand((N, K), generator=gen, device="cuda") * 2 - 1).to(dt)
        odt = torch.bfloat16 if dt == torch.float8_e4m3fn else dt
        out = torch.empty((M, N), dtype=odt, device="cuda")
        ref = A.float() @ W.float().t()
        bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
        s = torch.cuda.current_stream().cuda_stream
        din, dout = G.dtype_code(dt), G.dtype_code(odt)
        variants = {}
        if dt == torch.float8_e4m3fn:
            one = torch.ones((), device="cuda")
            variants["hipblaslt_scaled_mm"] = lambda: torch._scaled_mm(
                A, W.t(), scale_a=one, scale_b=one, out_dtype=odt)
        else:
            variants["hipblaslt_linear"] = lambda: torch.nn.functional.linear(A, W)
        for t in a.tiles.split(","):
            variants[f"unsplit[{t}]"] = (lambda t=t: G.gemm(A, W, out, tile=t, mode=mode,
                                                            ksplit=1))
        for S in (int(x) for x in a.splits.split(",")):
            if K % S or M % 256 or N % 256 or (K * A.element_size() // 128) % (2 * S):
                continue
            part = torch.empty((S, M, N), dtype=odt, device="cuda")
            ptrs = [part[j].data_ptr() for j in range(S)]

            def two(S=S, part=part, ptrs=ptrs):
                C.gemm(A.data_ptr(), W.data_ptr(), part.data_ptr(), K, K, N, M, N, K // S, din,
                       dout, G.TILES["pt4"], G.MODES[mode], 0, 0, 0, 0, s, 0, S)
                C.reduce_sum(out.data_ptr(), ptrs, M * N, dout, s)

            variants[f"ks{S}[pt4]/reduce"] = two
            if odt != torch.float32:
                p32 = torch.empty((S, M, N), dtype=torch.float32, device="cuda")
                q32 = [p32[j].data_ptr() for j in range(S)]

                def two32(S=S, p32=p32, q32=q32):
                    C.gemm(A.data_ptr(), W.data_ptr(), p32.data_ptr(), K, K, N, M, N, K // S,
                           din, G.DT_F32, G.TILES["pt4"], G.MODES[mode], 0, 0, 0, 0, s, 0, S)
                    C.reduce_sum(out.data_ptr(), q32, M * N, dout, s, G.DT_F32)

                variants[f"ks{S}[pt4]/reduce-f32"] = two32
        if a.only:
            variants = {k: v for k, v in variants.items() if re.search(a.only, k)}
        for k, fn in variants.items():
            if k.startswith("hipblaslt"):
                continue
            errs = []
            for _ in range(a.checks):
                out.fill_(float("nan"))
                fn()
                torch.cuda.synchronize()
                errs.append(float((out.float() - ref).abs().max()))
            err = max(errs)
            nbad = sum(e > bound for e in errs)
            print(f"  check {k:24s} max|err| {err:.4g} (bound {bound:.4g}) "
                  f"{'ok' if not nbad else f'FAIL in {nbad} of {a.checks}'}", flush=True)
        del ref
        times = {k: [] for k in variants}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for k, fn in variants.items():
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                ev0.record()
                for _ in range(a.iters):
                    fn()
                ev1.record()
                torch.cuda.synchronize()
                times[k].append(ev0.elapsed_time(ev1) / a.iters)
        flop = 2.0 * M * N * K
        print(f"\n{M}x{N}x{K} {a.dtype}: median ms over {a.rounds} rounds", flush=True)
        for k, ts in times.items():
            med = statistics.median(ts)
            print(f"  {k:24s} {med:8.4f} ms  {flop / med / 1e9:8.1f} TFLOP/s", flush=True)
        del A, W, out
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
