"""Which capture topology crashes hipStreamEndCapture? World-1 plans, no IPC, no peers.

The cs2 IPC pipeline (one peer's pulls split over two copy streams, joined by an event edge from
the second copy stream into the first) segfaults inside ``hipStreamEndCapture``
(``DDLB_GRAPH_DEBUG=1`` trace, profiles/r03/r3_13_*). Each variant below is captured, replayed
once and byte-checked in a child process of its own (a crash only ends that child):

* ``side_side``: memcpy on s1 and s2, edge s2 -> s1, edge s1 -> s0 (the cs2 shape)
* ``side_main``: memcpy on s1 and s2, edges s2 -> s0 and s1 -> s0 (no side-to-side edge)
* ``side_side_kernel``: as side_side with the s2 copy on CUs (a kernel node, not a memcpy node)
* ``side_side_tail``: as side_side, then one more memcpy on s1 after the edge
* ``cs2_exact``: the cs2 pipeline's op sequence (4 streams: prologue signal, READY waits on both
  copy streams, two stages of split copies + edges + GEMM, ACK signal, ACK wait) on local buffers,
  with the waited flags preset so every wait is already satisfied
* ``cs2_noedge``: cs2_exact with each stage's s3 -> s2 edge replaced by s3 -> s0
* ``cycle``: no signals at all, only copies and event edges s1 -> s2 then s2 -> s1 (a cycle of
  stream relations, no cycle of nodes): crashed hipStreamEndCapture; now refused by
  ``graph_capturable()`` (the child exits 1 with the refusal), the cs2 variants capture since the
  executor no longer joins wait-only streams before a cross-process wait

    python scripts/diag_graph_edges.py            # every variant, one child each
"""

from __future__ import annotations

import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = ["side_main", "side_side_kernel", "side_side_tail", "side_side", "cs2_noedge",
            "cs2_exact", "cycle"]
NB = 1 << 20


def build_cs2(variant: str):
    from ddlb_amd.parallel.plan import COPY_ENGINE, DT_BF16, SIG_KERNEL, Plan

    plan = Plan(0, 1, nstreams=4)
    src = plan.buffer("src", 4 * NB)
    dst = plan.buffer("dst", 4 * NB)
    a = plan.buffer("a", 256 * 256 * 2)
    b = plan.buffer("b", 256 * 256 * 2)
    c = plan.buffer("c", 256 * 256 * 2)
    fin = plan.buffer("fin", 64)    # preset: every wait already satisfied
    fout = plan.buffer("fout", 64)  # signal targets
    plan.signal(0, [fout], method=SIG_KERNEL)
    plan.wait_signal(2, [fin], method=SIG_KERNEL)
    plan.wait_signal(3, [fin + 4], method=SIG_KERNEL)
    for j in range(2):
        plan.copy(2, dst + 2 * j * NB, src + 2 * j * NB, NB, method=COPY_ENGINE)
        plan.copy(3, dst + (2 * j + 1) * NB, src + (2 * j + 1) * NB, NB, method=COPY_ENGINE)
        plan.edge(3, 0 if variant == "cs2_noedge" else 2)
        plan.edge(2, 0)
        plan.gemm(0, a, b, c, M=256, N=256, K=256, lda=256, ldb=256, ldc=256, din=DT_BF16,
                  dout=DT_BF16)
    plan.signal(2, [fout + 4], method=SIG_KERNEL)
    plan.wait_signal(0, [fin + 8], method=SIG_KERNEL)
    return plan


def build(variant: str):
    from ddlb_amd.parallel.plan import COPY_ENGINE, COPY_KERNEL, Plan

    if variant.startswith("cs2"):
        return build_cs2(variant)

    plan = Plan(0, 1, nstreams=3)
    src = plan.buffer("src", 3 * NB)
    dst = plan.buffer("dst", 3 * NB)
    if variant == "cycle":
        plan.copy(1, dst, src, NB, method=COPY_ENGINE)
        plan.edge(1, 2)
        plan.copy(2, dst + NB, src + NB, NB, method=COPY_ENGINE)
        plan.edge(2, 1)
        plan.copy(1, dst + 2 * NB, src + 2 * NB, NB, method=COPY_ENGINE)
        plan.edge(1, 0)
        plan.edge(2, 0)
        return plan
    plan.copy(1, dst, src, NB, method=COPY_ENGINE)
    plan.copy(2, dst + NB, src + NB, NB,
              method=COPY_KERNEL if variant == "side_side_kernel" else COPY_ENGINE)
    if variant == "side_main":
        plan.edge(2, 0)
    else:
        plan.edge(2, 1)
    if variant == "side_side_tail":
        plan.copy(1, dst + 2 * NB, src + 2 * NB, NB, method=COPY_ENGINE)
    plan.edge(1, 0)
    return plan


def child(variant: str) -> int:
    import torch

    from ddlb_amd.ops import load

    C = load()
    plan = build(variant)
    bufs = {"src": torch.randint(0, 255, (4 * NB,), dtype=torch.uint8, device="cuda"),
            "dst": torch.zeros(4 * NB, dtype=torch.uint8, device="cuda"),
            "a": torch.zeros(256 * 256, dtype=torch.bfloat16, device="cuda"),
            "b": torch.zeros(256 * 256, dtype=torch.bfloat16, device="cuda"),
            "c": torch.zeros(256 * 256, dtype=torch.bfloat16, device="cuda"),
            "fin": torch.full((16,), 0x7FFFFFF0, dtype=torch.int32, device="cuda"),
            "fout": torch.zeros(16, dtype=torch.int32, device="cuda")}
    ex = C.PlanExecutor(0, plan.nstreams, max(plan.nevents, 1), list(plan.stream_priority))
    ex.load(plan.encode(lambda ref: bufs[ref.buf].data_ptr() + ref.off))
    ex.enable_graph(True)
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        bufs["dst"].zero_()
        ex.run(stream)
        torch.cuda.synchronize()
    n = {"side_side_tail": 3 * NB, "cycle": 3 * NB}.get(
        variant, 4 * NB if variant.startswith("cs2") else 2 * NB)
    ok = torch.equal(bufs["dst"][:n], bufs["src"][:n])
    print(f"{variant}: replayed, bytes {'ok' if ok else 'WRONG'}", flush=True)
    return 0 if ok else 1


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    rc = 0
    for v in VARIANTS:
        r = subprocess.run([sys.executable, "-u", __file__, "--child", v], capture_output=True,
                           text=True, timeout=120)
        out = (r.stdout + r.stderr).strip().splitlines()
        tail = [x for x in out if x.startswith(v) or "[graph]" in x and "op " not in x][-3:]
        print(f"{v}: exit {r.returncode}  " + " | ".join(tail), flush=True)
        rc |= r.returncode != 0
    return int(rc)


if __name__ == "__main__":
    sys.exit(main())
