"""Do hipGraph replays run independent branches concurrently on this ROCm? Capture two
branches (forked onto a side stream inside the capture) that each spin ~2 ms, replay, and compare
with one branch alone: ~2 ms = concurrent branches, ~4 ms = the graph was serialized."""
import time

import torch


def main():
    torch.cuda.init()
    # calibrate torch.cuda._sleep
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(1 << 22)
    e1.record()
    torch.cuda.synchronize()
    cyc = int((1 << 22) * 2.0 / e0.elapsed_time(e1))  # ~2 ms
    for branches in (1, 2, 4):
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        sides = [torch.cuda.Stream() for _ in range(branches - 1)]
        with torch.cuda.graph(g, stream=cap):
            fork = torch.cuda.Event()
            fork.record(cap)
            joins = []
            for s in sides:
                s.wait_event(fork)
                with torch.cuda.stream(s):
                    torch.cuda._sleep(cyc)
                    j = torch.cuda.Event()
                    j.record(s)
                    joins.append(j)
            torch.cuda._sleep(cyc)
            for j in joins:
                cap.wait_event(j)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / 5
        print(f"graph with {branches} concurrent 2-ms branches: {ms:.2f} ms per replay")


if __name__ == "__main__":
    main()
