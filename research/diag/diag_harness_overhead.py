"""Where the reference-default timing's per-iteration overhead goes (VERDICT r3 weak #8:
``harness_mean_ms`` 0.1137 vs a 0.0999 ms back-to-back window at world 1).

One iteration of the reference's default mode (``ddlb/benchmark.py:161-172``) is
``barrier(); t0; run(); synchronize(); t1``. Measured here, per iteration (median of N):

* ``sync``       t0; synchronize(); t1 on an idle device (the completion-wait floor);
* ``tiny``       one 64-thread kernel launched on an idle device, then synchronize();
* ``run``        the flagship primitive's run() + synchronize() (harness mode);
* ``window``     K back-to-back run() calls inside one sync pair, per call (the bench window);
* ``enqueue``    host time of run() alone (the call returns after the launch);

under the HIP device scheduling flag given by ``--schedule`` (auto | spin | yield | blocking),
set with ``hipSetDeviceFlags`` BEFORE torch creates the context (a fresh process per flag).

    python research/diag/diag_harness_overhead.py [--schedule auto,spin] [-n 200]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}


def child(schedule: str, n: int) -> dict:
    if schedule != "auto":
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[schedule]))
        if rc != 0:
            return {"error": f"hipSetDeviceFlags({schedule}) = {rc}"}
    import socket

    import torch

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["DDLB_CHILD_INIT_METHOD"] = f"tcp://127.0.0.1:{s.getsockname()[1]}"
    s.close()
    from ddlb_amd.communicator import Communicator
    from ddlb_amd.ops import load
    from ddlb_amd.primitives.tp_columnwise.native import NativeTPColumnwise

    comm = Communicator()
    comm.ensure_process_group()
    C = load()
    impl = NativeTPColumnwise(m=65536, n=1024, k=1024, dtype="bfloat16")
    tiny_src = torch.zeros(16, dtype=torch.uint8, device="cuda")
    tiny_dst = torch.zeros(16, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    def med(fn):
        xs = []
        for _ in range(n):
            comm.barrier()
            t0 = time.perf_counter()
            fn()
            xs.append((time.perf_counter() - t0) * 1e6)
        return statistics.median(xs)

    for _ in range(50):
        impl.run()
    torch.cuda.synchronize()
    out = {"schedule": schedule}
    out["sync_us"] = med(torch.cuda.synchronize)
    out["tiny_us"] = med(lambda: (C.copy(tiny_dst.data_ptr(), tiny_src.data_ptr(), 16, 1, stream),
                                  torch.cuda.synchronize()))
    out["run_us"] = med(lambda: (impl.run(), torch.cuda.synchronize()))
    enq = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        impl.run()
        enq.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    out["enqueue_us"] = statistics.median(enq)
    k = 50
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        impl.run()
    torch.cuda.synchronize()
    out["window_us"] = (time.perf_counter() - t0) * 1e6 / k
    impl.close()
    comm.destroy()
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedule", default="auto,spin,yield,blocking")
    ap.add_argument("-n", type=int, default=200)
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        print(json.dumps(child(a.child, a.n)), flush=True)
        return 0
    for sch in a.schedule.split(","):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", sch, "-n",
                            str(a.n)], capture_output=True, text=True, timeout=300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if not lines:
            print(f"{sch}: failed rc={r.returncode} {r.stderr[-400:]}", flush=True)
            continue
        d = json.loads(lines[-1])
        print("  ".join(f"{k} {v:.1f}" if isinstance(v, float) else f"{k} {v}"
                        for k, v in d.items()), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
