"""Do streams share HIP hardware queues (GPU_MAX_HW_QUEUES)? A busy side stream must not delay
the GEMM stream. Streams 1..S-1 each run a ~20 ms spin kernel; stream 0 runs 20 GEMMs; report
when stream 0 finishes. Run with different GPU_MAX_HW_QUEUES values (set before HIP init)."""
import os
import sys
import time

import torch


def main():
    nside = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda")
    A = torch.randn(16384, 1024, device=dev, dtype=torch.bfloat16)
    W = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    main_s = torch.cuda.Stream()
    sides = [torch.cuda.Stream() for _ in range(nside)]
    for _ in range(3):
        with torch.cuda.stream(main_s):
            torch.nn.functional.linear(A, W)
    torch.cuda.synchronize()
    # calibrate the spin: ~20 ms
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(1 << 24)
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / (1 << 24)
    cycles = int(20.0 / per)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in sides:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    done = torch.cuda.Event()
    with torch.cuda.stream(main_s):
        for _ in range(20):
            torch.nn.functional.linear(A, W)
        done.record()
    done.synchronize()
    t_main = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) * 1e3
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'unset')} side_streams={nside}: "
          f"GEMM stream done after {t_main:.1f} ms (alone ~1 ms), all done {t_all:.1f} ms")


if __name__ == "__main__":
    main()
