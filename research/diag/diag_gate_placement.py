"""Why a flag-gated persistent GEMM needs its CU reserve (MIN_GATE_RESERVE's cause).

Hypothesis: the workgroup dispatcher places a kernel's workgroups on shader arrays (SAs) in turn
and does not move a workgroup to another SA when its SA has no room, so a feeding kernel (the
RCCL collective, a copy / signal kernel) blocks as soon as ONE of its workgroups is assigned to an
SA whose every CU holds a spinning gated tile. A gated GEMM is then deadlock-free iff it leaves
at least one CU free in EVERY shader array: reserve >= number of SAs (MI355X: 8 XCDs x 4 SAs of
8 CUs = 32), with the gated workgroups spread evenly (the dispatcher's round-robin does that).
This matches every recorded point of profiles/r04/r4_33_*, r4_34_*, r4_36_*: grids of 232 / 240
(29 / 30 per XCD: some SA full) hung with feeders of >= 16-32 workgroups; 224 (28 per XCD, 7
per SA) ran with 8 to 64.

Each configuration runs in its own process (a hang there is a bounded spin: the gated tiles give
up after seconds and report it in the timeout word). Per run: the gated GEMM (grid
num_cus - reserve) is enqueued FIRST on a normal-priority stream; a copy kernel of ``blocks``
workgroups and then the signal kernel that raises the GEMM's flag follow on a high-priority stream
(the RCCL-fed fused plans' order). Reports the wall time and the timeout code, plus the device
topology from KFD's sysfs (shader engines / arrays per engine / CUs per array).

    python research/diag/diag_gate_placement.py --configs 32:32,32:64,32:256,24:8,24:32,16:16
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def kfd_topology():
    """Shader-array layout of the GPU (KFD sysfs where readable, else rocminfo; empty off-GPU)."""
    keys = ("simd_count", "array_count", "simd_arrays_per_engine", "cu_per_simd_array",
            "simd_per_cu", "num_xcc", "max_waves_per_simd", "lds_size_in_kb")
    out = []
    for path in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        props = {}
        try:
            with open(path) as fh:
                for line in fh:
                    k, _, v = line.strip().partition(" ")
                    if k in keys:
                        props[k] = int(v)
        except OSError:
            continue
        if props.get("simd_count", 0) > 0:
            out.append(props)
    if out:
        return out
    try:  # rocminfo: "Compute Unit", "Shader Engines", "Shader Arrs. per Eng." of each GPU agent
        r = subprocess.run(["rocminfo"], capture_output=True, text=True, timeout=60)
    except (OSError, subprocess.TimeoutExpired):
        return out
    cur = {}
    for line in r.stdout.splitlines():
        k, _, v = line.strip().partition(":")
        k, v = k.strip(), v.strip().split(" ")[0]
        if k in ("Compute Unit", "Shader Engines", "Shader Arrs. per Eng.", "SIMDs per CU"):
            cur[k] = int(v) if v.isdigit() else v
        if k == "Name" and v.startswith("gfx"):
            cur = {"name": v}
            out.append(cur)
    return [c for c in out if "Compute Unit" in c]


def one(reserve: int, blocks: int) -> dict:
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext
    from ddlb_amd.parallel.plan import DT_BF16, SIG_KERNEL, Plan

    comm = Communicator()
    comm.ensure_process_group()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    M, N, K = 256 * (cus - reserve), 256, 256  # one 256x256 tile per gated workgroup
    nbytes = 64 << 20
    plan = Plan(0, 1, nstreams=2, stream_priority=[0, 1])
    a = plan.buffer("a", M * K * 2)
    bt = plan.buffer("bt", N * K * 2)
    c = plan.buffer("c", M * N * 2)
    src = plan.buffer("src", nbytes)
    dst = plan.buffer("dst", nbytes)
    fl = plan.buffer("flags", 256, zero=True)
    plan.gemm(0, a, bt, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, din=DT_BF16, dout=DT_BF16, tile=19,
              flags=fl, flag_rows=M, nshards=1, tile_order=1, reserve_cus=reserve)
    plan.copy_multi(1, [(dst, src, nbytes)], max_blocks=blocks)
    plan.signal(1, [fl], method=SIG_KERNEL)
    ctx = NativeContext(comm)
    bound = ctx.bind(plan)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bound.run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    code = int(bound.ex.read_timeout())
    bound.close()
    ctx.close()
    return {"reserve": reserve, "gemm_grid": (cus - reserve) // 8 * 8, "feeder_blocks": blocks,
            "ms": round(ms, 2), "timeout": code}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="32:32,32:64,32:256,24:8,24:32,16:16")
    p.add_argument("--one", default=None, help=argparse.SUPPRESS)
    a = p.parse_args()
    if a.one:
        r, b = (int(x) for x in a.one.split(":"))
        print(json.dumps(one(r, b)), flush=True)
        return 0
    print(json.dumps({"kfd_topology": kfd_topology()}), flush=True)
    for cfg in a.configs.split(","):
        # a blocked feeder shows as the gated tiles giving up: ~0.2 s per tile at 2^18 polls
        env = dict(os.environ, DDLB_CHILD_INIT_METHOD=f"tcp://127.0.0.1:{_free_port()}",
                   DDLB_SPIN_LIMIT=str(1 << 18))
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            env.pop(k, None)
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", cfg],
                               capture_output=True, text=True, timeout=90, env=env)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(lines[-1] if lines else json.dumps({"config": cfg, "rc": r.returncode,
                                                      "err": r.stderr[-400:]}), flush=True)
        except subprocess.TimeoutExpired:
            print(json.dumps({"config": cfg, "error": "timeout 90 s"}), flush=True)
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
