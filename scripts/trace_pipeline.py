"""Stage-level trace of one native pipeline (per-op roctx ranges from the C++ executor).

Every op of the plan is enqueued inside a roctx range named by ``Plan.labels()`` ("gemm s3",
"copy p1 b2", "wait_signal flags+8", ...), so under

    rocprofv3 --marker-trace --kernel-trace --kernel-rename --stats -d OUT -- \\
        python3 scripts/trace_pipeline.py --algorithm coll_pipeline --backend ipc -s 4

the kernel trace names each GEMM / copy / signal kernel by its stage. Launch one process per rank
(RANK / WORLD_SIZE / MASTER_* in the environment; ranks may share one GPU with
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo for IPC plans).
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--primitive", default="tp_columnwise", choices=["tp_columnwise", "tp_rowwise"])
    p.add_argument("-m", type=int, default=16384)
    p.add_argument("-n", type=int, default=1024)
    p.add_argument("-k", type=int, default=1024)
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--algorithm", default="coll_pipeline")
    p.add_argument("--backend", default="ipc")
    p.add_argument("-s", type=int, default=4)
    p.add_argument("--opts", default="{}", help="extra native options (JSON)")
    p.add_argument("--runs", type=int, default=5)
    a = p.parse_args()
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.primitives.registry import resolve

    comm = Communicator()
    comm.ensure_process_group()
    opts = dict(algorithm=a.algorithm, backend=a.backend, s=a.s, trace=True, graph=False,
                **json.loads(a.opts))
    cls, opts, _ = resolve(a.primitive, "native", opts)
    impl = cls(m=a.m, n=a.n, k=a.k, dtype=a.dtype, **opts)
    for _ in range(a.runs):
        out = impl.run()
    torch.cuda.synchronize()
    impl.validate(out)
    if comm.rank == 0:
        print("plan ops:", json.dumps(impl.plan.labels()))
        print("trace ok")
    impl.close()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
