"""Host-side overhead of one primitive run() in the reference's default timing mode
(device sync + barrier before every iteration, perf_counter around run()+sync).

A tiny shape makes GPU time negligible, so the number is launch/enqueue latency:
native plan executor (eager and hipGraph replay) vs the pytorch slot vs a bare torch.matmul.
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import socket

    import torch

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["DDLB_CHILD_INIT_METHOD"] = f"tcp://127.0.0.1:{s.getsockname()[1]}"
    s.close()
    from ddlb_amd.communicator import Communicator
    from ddlb_amd.primitives.registry import resolve

    comm = Communicator()
    comm.ensure_process_group()
    shapes = [(1024, 1024, 1024), (65536, 1024, 1024)]
    variants = [("native eager", "native", {"algorithm": "coll_pipeline", "s": 4}),
                ("native graph", "native", {"algorithm": "coll_pipeline", "s": 4, "graph": True}),
                ("native default", "native", {"algorithm": "default"}),
                ("pytorch", "pytorch", {"empty_cache": False})]
    for (m, n, k) in shapes:
        print(f"\nshape m={m} n={n} k={k}")
        for label, impl_name, opts in variants:
            cls, o, _ = resolve("tp_columnwise", impl_name, opts)
            impl = cls(m=m, n=n, k=k, dtype="bfloat16", **o)
            ts = []
            for i in range(60):
                comm.barrier()
                t0 = time.perf_counter()
                impl.run()
                comm.synchronize()
                ts.append((time.perf_counter() - t0) * 1e6)
            ts = ts[10:]
            print(f"  {label:16s} median {statistics.median(ts):8.1f} us   min {min(ts):8.1f} us")
            impl.close()
    comm.destroy()


if __name__ == "__main__":
    main()
