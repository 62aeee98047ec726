"""Worker for tests/test_native_gpu.py::test_gemm_first_queue_pools (run with its own
GPU_MAX_HW_QUEUES, which HIP reads once per process).

A flag-gated persistent GEMM is enqueued on stream 0 BEFORE the signal kernel that raises its
flags on stream 1 (the RCCL-fed fused plans' ``gemm_first`` order). If the two streams share one
in-order hardware queue, the signal waits behind the spinning tiles until their bounded spin
gives up (the timeout word is set); on separate queues the GEMM completes at once. Prints one
JSON line: {"prio": [p0, p1], "timeout": code, "ms": wall, "err": max|err|}.
"""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext
    from ddlb_amd.parallel.plan import DT_BF16, SIG_KERNEL, Plan

    prio = [int(x) for x in os.environ["DDLB_TEST_PRIO"].split(",")]
    comm = Communicator()
    comm.ensure_process_group()
    M, N, K = 4096, 512, 256
    plan = Plan(0, 1, nstreams=2, stream_priority=prio)
    a = plan.buffer("a", M * K * 2)
    bt = plan.buffer("bt", N * K * 2)
    c = plan.buffer("c", M * N * 2)
    fl = plan.buffer("flags", 256, zero=True)
    plan.gemm(0, a, bt, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, din=DT_BF16, dout=DT_BF16,
              tile=19, flags=fl, flag_rows=M // 2, nshards=2, tile_order=1, reserve_cus=32)
    plan.signal(1, [fl, fl + 4], method=SIG_KERNEL)
    ctx = NativeContext(comm)
    bound = ctx.bind(plan)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    bound.buffer("a").view(torch.bfloat16).view(M, K).copy_(A)
    bound.buffer("bt").view(torch.bfloat16).view(N, K).copy_(W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        bound.run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    out = bound.buffer("c").view(torch.bfloat16).view(M, N).float()
    err = float((out - A.float() @ W.float().T).abs().max())
    code = bound.ex.read_timeout()
    bound.close()
    ctx.close()
    print(json.dumps({"prio": prio, "timeout": int(code), "ms": ms, "err": err}), flush=True)


if __name__ == "__main__":
    main()
