"""Time the native d-way reduce kernel (reduce-scatter's sum) on local HBM.

    python scripts/bench_reduce.py                          # fixed-count unrolled kernels
    DDLB_REDUCE_GENERIC=1 python scripts/bench_reduce.py    # runtime-count kernel (A/B)

Prints one line per source count: time and effective bandwidth (nsrc reads + 1 write).
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddlb_amd.ops import load  # noqa: E402


def main() -> None:
    C = load()
    count = 1 << 26  # 64 Mi bf16 = 128 MiB per source
    kind = "generic" if os.environ.get("DDLB_REDUCE_GENERIC") else "fixed"
    s = torch.cuda.current_stream().cuda_stream
    for nsrc in (2, 4, 8):
        srcs = [torch.randn(count, device="cuda", dtype=torch.bfloat16) for _ in range(nsrc)]
        out = torch.empty(count, device="cuda", dtype=torch.bfloat16)
        ptrs = [t.data_ptr() for t in srcs]
        for _ in range(5):
            C.reduce_sum(out.data_ptr(), ptrs, count, 2, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 20
        e0.record()
        for _ in range(iters):
            C.reduce_sum(out.data_ptr(), ptrs, count, 2, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        gbs = (nsrc + 1) * count * 2 / (ms * 1e-3) / 1e9
        print(f"reduce[{kind}] nsrc={nsrc} count={count} bf16: {ms * 1e3:.1f} us, {gbs:.0f} GB/s",
              flush=True)
        del srcs, out


if __name__ == "__main__":
    main()
