"""Time the native d-way reduce kernel (reduce-scatter's sum) on local HBM.

    python scripts/bench_reduce.py                          # fixed-count unrolled kernels
    DDLB_REDUCE_GENERIC=1 python scripts/bench_reduce.py    # runtime-count kernel (A/B)
    python scripts/bench_reduce.py --copy                   # CU copy kernel, 7 segments
    DDLB_COPY_NT=1 python scripts/bench_reduce.py --copy    # with non-temporal loads (A/B)

Prints one line per source count: time and effective bandwidth (nsrc reads + 1 write).
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddlb_amd.ops import load  # noqa: E402


def bench_copy(C) -> None:
    """The IPC all-gather's CU copy: 7 segments (one per peer at d=8) of 16 MiB each."""
    kind = "nt-load" if os.environ.get("DDLB_COPY_NT") else "plain"
    s = torch.cuda.current_stream().cuda_stream
    seg = 16 << 20
    src = torch.empty(7 * seg, device="cuda", dtype=torch.uint8).random_()
    dst = torch.empty_like(src)
    segs = [(dst.data_ptr() + i * seg, src.data_ptr() + i * seg, seg) for i in range(7)]
    for blocks in (128, 512, 2048):
        for _ in range(5):
            C.copy_multi(segs, blocks, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            C.copy_multi(segs, blocks, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        assert torch.equal(src, dst)
        print(f"copy[{kind}] 7 x 16 MiB blocks={blocks}: {ms * 1e3:.1f} us, "
              f"{2 * 7 * seg / (ms * 1e-3) / 1e9:.0f} GB/s", flush=True)


def main() -> None:
    C = load()
    if "--copy" in sys.argv:
        bench_copy(C)
        return
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
