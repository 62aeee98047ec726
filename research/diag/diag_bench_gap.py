"""Where does bench.py's world-1 step time go? Times, in one process, 50-step loops of:
impl.run() (the bench path), the bare GEMM on the impl's own buffers, and torch.matmul,
with perf_counter+sync (bench.py's clock) and with events."""
import os
import socket
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["DDLB_CHILD_INIT_METHOD"] = f"tcp://127.0.0.1:{s.getsockname()[1]}"
    s.close()
    from ddlb_amd.communicator import Communicator
    from ddlb_amd.ops.gemm import gemm
    from ddlb_amd.primitives.registry import resolve

    comm = Communicator()
    comm.ensure_process_group()
    m, n, k = 65536, 1024, 1024
    cls, o, _ = resolve("tp_columnwise", "native", {"algorithm": "default"})
    impl = cls(m=m, n=n, k=k, dtype="bfloat16", **o)
    A = impl.bound.view(impl.io.a)
    W = impl.bound.view(impl.io.b)
    C = impl.out
    A2 = (torch.rand((m, k), device="cuda") * 2 - 1).bfloat16()
    W2 = (torch.rand((n, k), device="cuda") * 2 - 1).bfloat16()
    C2 = torch.empty((m, n), device="cuda", dtype=torch.bfloat16)
    print("A", tuple(A.shape), A.stride(), "W", tuple(W.shape), W.stride(), "C", tuple(C.shape))
    variants = {
        "impl.run": lambda: impl.run(),
        "gemm(impl bufs) auto": lambda: gemm(A, W, C),
        "gemm(impl bufs) pt4": lambda: gemm(A, W, C, tile="pt4"),
        "gemm(fresh bufs) auto": lambda: gemm(A2, W2, C2),
        "gemm(fresh bufs) pt4": lambda: gemm(A2, W2, C2, tile="pt4"),
        "torch.matmul": lambda: torch.matmul(A2, W2.t(), out=C2),
    }
    res = {kname: ([], []) for kname in variants}
    for rnd in range(5):
        for name, fn in variants.items():
            for _ in range(10):
                fn()
            comm.barrier()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            res[name][0].append((t1 - t0) * 1e3 / 50)
            res[name][1].append(e0.elapsed_time(e1) / 50)
    for name, (wall, ev) in res.items():
        print(f"{name:26s} wall {statistics.median(wall)*1e3:8.1f} us  events "
              f"{statistics.median(ev)*1e3:8.1f} us   (min wall {min(wall)*1e3:.1f})")
    impl.close()
    comm.destroy()


if __name__ == "__main__":
    main()
