"""Print (and optionally simulate) the native plan of a primitive/algorithm for one rank.

    python -m ddlb_amd.parallel.explain --primitive tp_columnwise -d 8 -m 65536 -n 1024 \
        -k 1024 --algorithm p2p_pipeline --backend ipc --rank 0
    python -m ddlb_amd.parallel.explain ... --simulate   # CPU run of all d ranks (small shapes)

The simulation executes every rank's plan on the CPU with the race / deadlock checker
(:mod:`ddlb_amd.parallel.sim`) — the same check the test-suite runs for every algorithm.
"""

from __future__ import annotations

import argparse

from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise, build_tp_rowwise
from ddlb_amd.parallel.plan import NAME_DT, SIG_KERNEL, SIG_STREAM


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--primitive", default="tp_columnwise", choices=["tp_columnwise", "tp_rowwise"])
    p.add_argument("-d", "--world", type=int, default=2)
    p.add_argument("--rank", type=int, default=0)
    p.add_argument("-m", type=int, default=64)
    p.add_argument("-n", type=int, default=16)
    p.add_argument("-k", type=int, default=32)
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--algorithm", default="default")
    p.add_argument("--backend", default="rccl")
    p.add_argument("--order", default="AG_before")
    p.add_argument("-s", type=int, default=2)
    p.add_argument("--protocol", default="memcpy")
    p.add_argument("--signal", default="stream", choices=["stream", "kernel"])
    p.add_argument("--no-ring", action="store_true")
    p.add_argument("--fused", action="store_true")
    p.add_argument("--simulate", action="store_true")
    a = p.parse_args(argv)
    cfg = AlgoConfig(algorithm=a.algorithm, backend=a.backend, order=a.order, s=a.s,
                     ring=not a.no_ring, protocol=a.protocol,
                     signal=SIG_STREAM if a.signal == "stream" else SIG_KERNEL, fused=a.fused)
    din = NAME_DT[a.dtype]
    dout = NAME_DT["bfloat16"] if a.dtype == "float8_e4m3fn" else din
    build = build_tp_columnwise if a.primitive == "tp_columnwise" else build_tp_rowwise
    plan, io = build(a.rank, a.world, a.m, a.n, a.k, din, dout, cfg)
    print(plan.describe())
    print(f"  inputs: A={io.a}  B={io.b}\n  output: {io.out}")
    if a.simulate:
        import torch

        from ddlb_amd.parallel.sim import Simulator, make_buffers, read_tensor, write_tensor

        built = [build(r, a.world, a.m, a.n, a.k, din, dout, cfg) for r in range(a.world)]
        bufs = make_buffers([b[0] for b in built])
        g = torch.Generator().manual_seed(0)
        A = torch.randint(-2, 3, (a.m, a.k), generator=g).float()
        B = torch.randint(-2, 3, (a.k, a.n), generator=g).float()
        tdt = read_tensor(bufs[0], built[0][1].a).dtype
        for r, (_, rio) in enumerate(built):
            if a.primitive == "tp_columnwise":
                ml = a.m // a.world
                write_tensor(bufs[r], rio.a, A[r * ml:(r + 1) * ml].to(tdt))
                write_tensor(bufs[r], rio.b, B.t().contiguous().to(tdt))
            else:
                kl = a.k // a.world
                write_tensor(bufs[r], rio.a, A[:, r * kl:(r + 1) * kl].contiguous().to(tdt))
                write_tensor(bufs[r], rio.b, B[r * kl:(r + 1) * kl].t().contiguous().to(tdt))
        sim = Simulator([b[0] for b in built], bufs)
        for _ in range(3):
            sim.run_epoch()
        ref = A @ B
        worst = 0.0
        for r, (_, rio) in enumerate(built):
            out = read_tensor(bufs[r], rio.out).float()
            want = ref if a.primitive == "tp_columnwise" else ref[
                r * (a.m // a.world):(r + 1) * (a.m // a.world)]
            worst = max(worst, float((out - want).abs().max()))
        print(f"simulated {a.world} ranks x 3 epochs: no race, no deadlock, max|err| = {worst}")


if __name__ == "__main__":
    main()
