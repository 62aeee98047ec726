"""Which hipBLASLt kernel does torch pick for the flagship GEMM, per call form? (rocprof target)"""
import statistics
import sys

import torch


def main():
    m, n, k = 65536, 1024, 1024
    A = (torch.rand((m, k), device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand((n, k), device="cuda") * 2 - 1).bfloat16()
    C = torch.empty((m, n), device="cuda", dtype=torch.bfloat16)
    forms = {
        "matmul(A, W.t())": lambda: torch.matmul(A, W.t()),
        "matmul(A, W.t(), out=C)": lambda: torch.matmul(A, W.t(), out=C),
        "F.linear(A, W)": lambda: torch.nn.functional.linear(A, W),
        "mm(A, W.t())": lambda: torch.mm(A, W.t()),
    }
    res = {f: [] for f in forms}
    for _ in range(5):
        for name, fn in forms.items():
            for _ in range(5):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / 50)
    for name, t in res.items():
        print(f"{name:28s} {statistics.median(t)*1e3:8.1f} us")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
