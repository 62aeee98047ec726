"""Head-of-line blocking check for the plan executor's streams: side streams blocked on a
hipStreamWaitValue32 (flag released by the host after 60 ms) must not delay GEMMs on the main
stream. The main stream's completion is observed through a signal into pinned host memory."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from ddlb_amd.ops import load
    from ddlb_amd.parallel.plan import DT_BF16, SIG_STREAM, Plan, Ref

    C = load()
    nside = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    m, n, k = 16384, 1024, 1024
    A = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    flag = torch.zeros(64, dtype=torch.int32, pin_memory=True)
    done = torch.zeros(64, dtype=torch.int32, pin_memory=True)
    plan = Plan(0, 1, nstreams=1 + nside, stream_priority=[0] + [1] * nside)
    for s in range(1, nside + 1):
        plan.wait_signal(s, [Ref("flag")], method=SIG_STREAM)
    for _ in range(20):
        plan.gemm(0, Ref("A"), Ref("W"), Ref("C"), M=m, N=n, K=k, lda=k, ldb=k, ldc=n,
                  din=DT_BF16, dout=DT_BF16)
    plan.signal(0, [Ref("done")], method=SIG_STREAM)
    addr = {"A": A.data_ptr(), "W": W.data_ptr(), "C": out.data_ptr(), "flag": flag.data_ptr(),
            "done": done.data_ptr()}
    ex = C.PlanExecutor(0, plan.nstreams, max(plan.nevents, 1), list(plan.stream_priority))
    ex.load(plan.encode(lambda r: addr[r.buf] + r.off))
    stream = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ex.run(stream)
    t_done = None
    while time.perf_counter() - t0 < 0.060:
        if t_done is None and int(done[0]) >= 1:
            t_done = (time.perf_counter() - t0) * 1e3
    flag[0] = 1
    torch.cuda.synchronize()
    if t_done is None and int(done[0]) >= 1:
        t_done = float("nan")
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'unset')} blocked side "
          f"streams={nside}: main-stream GEMMs done after "
          f"{'>60 ms (blocked)' if t_done is None or t_done != t_done else f'{t_done:.2f} ms'}")


if __name__ == "__main__":
    main()
