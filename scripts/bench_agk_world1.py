"""In-kernel all-gather on one GPU: the flagship GEMM (m=65536 n=1024 k=1024 bf16) with the
copy workgroups pulling (np-1)/np of A from a local stand-in for the peers' memory (HBM instead of
xGMI), against the plain pt4 GEMM. Shows what the copy role and the flag gates cost and how much
of the copy hides under the GEMM.

    python scripts/bench_agk_world1.py [--np 8] [--nsub 8] [--ctas 32,64] [--iters 50]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(M, N, K, npro, nsub, ctas, gated=True, unit_kb=256, mode=0):
    from ddlb_amd.parallel.plan import DT_BF16, Plan, SIG_IN_LAUNCH, SIG_KERNEL

    rows = M // (npro * nsub)
    plan = Plan(0, 1, nstreams=1, stream_priority=[0])
    a = plan.buffer("a", M * K * 2)
    peer = plan.buffer("peer", M * K * 2)
    bt = plan.buffer("bt", N * K * 2)
    c = plan.buffer("c", M * N * 2)
    fl = plan.buffer("flags", 1024, zero=True)
    READY, ACK, ARRIVE, CNT = fl, fl + 128, fl + 256, fl + 512
    if not gated:
        plan.gemm(0, a, bt, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, din=DT_BF16, dout=DT_BF16,
                  tile=19)
        return plan
    plan.signal(0, [READY + 4 * p for p in range(1, npro)], method=SIG_KERNEL)
    plan.signal(0, [ARRIVE + 4 * j for j in range(nsub)], method=SIG_KERNEL)
    seg = rows * K * 2
    ag = dict(ctas=ctas, parts=max(1, seg // (unit_kb << 10)), rank=0,
              src=[a] + [peer] * (npro - 1), ack=[ACK + 4 * p for p in range(npro)],
              ready=READY, count=CNT, mode=mode,
              wait_acks=[ACK + 4 * p for p in range(npro)] if mode & 16 else None)
    plan.gemm(0, a, bt, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, din=DT_BF16, dout=DT_BF16,
              tile=19, flags=ARRIVE, flag_rows=rows, nshards=npro * nsub, nsub=nsub,
              first_shard=0, tile_order=1, ag=ag)
    plan.wait_signal(0, [ACK + 4 * p for p in range(1, npro)],
                     method=SIG_IN_LAUNCH if mode & 16 else SIG_KERNEL)
    return plan


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext

    ap = argparse.ArgumentParser()
    ap.add_argument("--np", type=int, default=8)
    ap.add_argument("--nsub", type=int, default=8)
    ap.add_argument("--ctas", default="32,64")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--unit-kb", default="256", help="copy unit sizes (KiB) to try")
    ap.add_argument("--modes", default="0",
                    help="ag_mode bit sets to try (csrc/gemm/gemm.h AgMode: 1 legacy plain "
                         "stores + release fence, 2 agent-scope gate acquire, 4 16 loads/lane)")
    a = ap.parse_args()
    M, N, K = 65536, 1024, 1024
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    os.environ.setdefault("DDLB_CHILD_INIT_METHOD", f"tcp://127.0.0.1:{sk.getsockname()[1]}")
    sk.close()
    comm = Communicator()
    comm.ensure_process_group()
    ctx = NativeContext(comm)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    ref = A.float() @ W.float().T
    own = M // a.np
    variants = [("pt4 GEMM only", 0, False, 0, 0)] + [
        (f"agk ctas={c} unit={u}K mode={md}", int(c), True, int(u), int(md))
        for c in a.ctas.split(",") for u in a.unit_kb.split(",") for md in a.modes.split(",")]
    for label, ctas, gated, unit, mode in variants:
        bound = ctx.bind(build(M, N, K, a.np, a.nsub, ctas, gated, unit or 256, mode))
        bound.enable_graph(True)
        av = bound.buffer("a").view(torch.bfloat16).view(M, K)
        av.copy_(A)
        if gated:
            av[own:].fill_(float("nan"))
            bound.buffer("peer").view(torch.bfloat16).view(M, K).copy_(A)
        bound.buffer("bt").view(torch.bfloat16).view(N, K).copy_(W)
        for _ in range(300 if not gated else 20):  # the first variant also ramps the clock
            bound.run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            bound.run()
        e1.record()
        torch.cuda.synchronize()
        bound.check_health()
        if gated:  # one more run from poisoned peer rows: this run's copies must land
            av[own:].fill_(float("nan"))
            bound.run()
            torch.cuda.synchronize()
            bound.check_health()
        out = bound.buffer("c").view(torch.bfloat16).view(M, N).float()
        err = (out - ref).abs().max().item()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"{label:>34}: {ms * 1e3:7.1f} us/run  {2 * M * N * K / ms / 1e9:7.0f} TFLOP/s  "
              f"copied {(M - own) * K * 2 / 2**20 if gated else 0:.0f} MiB  max|err| {err:.3f}",
              flush=True)
        bound.close()
    ctx.close()


if __name__ == "__main__":
    main()
