"""hipGraph replay of a plan with more streams than hardware queues (9 streams: 8 side-stream
copies + the caller's GEMM, joined), in one process. Run under different GPU_MAX_HW_QUEUES."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext
    from ddlb_amd.parallel.plan import DT_BF16, DT_F32, SIG_KERNEL, Plan

    comm = Communicator()
    comm.ensure_process_group()
    ctx = NativeContext(comm)
    nside, nb = 8, 1 << 20
    plan = Plan(0, 1, nstreams=1 + nside, stream_priority=[0] + [1] * nside)
    src = plan.buffer("src", nside * nb)
    dst = plan.buffer("dst", nside * nb)
    flags = plan.buffer("flags", 256, symmetric=True, zero=True)
    a = plan.buffer("a", 4096 * 1024 * 2)
    bt = plan.buffer("bt", 1024 * 1024 * 2)
    c = plan.buffer("c", 4096 * 1024 * 4)
    for i in range(nside):
        plan.copy(1 + i, dst + i * nb, src + i * nb, nb)
    plan.signal(1, [flags], method=SIG_KERNEL)
    plan.gemm(0, a, bt, c, M=4096, N=1024, K=1024, lda=1024, ldb=1024, ldc=1024, din=DT_BF16,
              dout=DT_F32)
    plan.wait_signal(0, [flags], method=SIG_KERNEL)
    bound = ctx.bind(plan)
    bound.enable_graph(True)
    x = torch.randint(0, 255, (nside * nb,), dtype=torch.uint8, device="cuda")
    bound.buffer("src")[:nside * nb].copy_(x)
    A = torch.randn(4096, 1024, device="cuda").bfloat16()
    W = torch.randn(1024, 1024, device="cuda").bfloat16()
    bound.buffer("a").view(torch.bfloat16).view(4096, 1024).copy_(A)
    bound.buffer("bt").view(torch.bfloat16).view(1024, 1024).copy_(W)
    for _ in range(5):
        bound.run()
    torch.cuda.synchronize()
    bound.check_health()
    assert torch.equal(bound.buffer("dst")[:nside * nb], x)
    out = bound.buffer("c").view(torch.float32).view(4096, 1024)
    torch.testing.assert_close(out, A.float() @ W.float().T, rtol=0, atol=1e-3 * 1024)
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')}: 9-stream plan "
          f"replayed 5x from a hipGraph, copies and GEMM correct, flag = "
          f"{int(bound.buffer('flags').view(torch.int32)[0])}")
    bound.close()
    ctx.close()
    comm.destroy()


if __name__ == "__main__":
    main()
