"""Native data-plane context: our RCCL communicator, IPC symmetric buffers, bound plans.

* :class:`NativeContext` — per-process; the RCCL ``ncclUniqueId`` and the IPC handles are exchanged
  over the control-plane process group (torch.distributed), the data plane never touches it.
* :class:`SymmetricBuffer` — one ``hipMalloc`` per rank, every peer's copy IPC-mapped (HIP IPC,
  dmabuf mode), exposed to torch through DLPack.
* :class:`BoundPlan` — a :class:`~ddlb_amd.parallel.plan.Plan` with its buffers allocated, its
  symbolic refs resolved to device addresses and loaded into a C++ ``PlanExecutor``; ``run()`` is
  a single native call that enqueues the whole schedule behind the caller's HIP stream.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional

from ddlb_amd.parallel.plan import DT_SIZE, OP_GEMM, RCCL_OPS, Plan, Ref
from ddlb_amd.parallel.sim import TORCH_DT


def graph_replay_supported() -> bool:
    """hipGraph replay segfaulted in this image's HIP runtime with GPU_MAX_HW_QUEUES = 1 or 2
    (a 9-stream plan replays fine with the default 4; profiles/r02/r2_17_*)."""
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) >= 4
    except ValueError:
        return True


def _raw_stream(device_index: int) -> int:
    """The caller's current HIP stream handle, without building a torch Stream object."""
    import torch

    getter = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if getter is not None:
        return getter(device_index)
    return torch.cuda.current_stream(device_index).cuda_stream


class SymmetricBuffer:
    def __init__(self, ctx: "NativeContext", nbytes: int, uncached: bool = False):
        import torch
        import torch.distributed as dist

        self.ctx = ctx
        self.nbytes = int(nbytes)
        C = ctx.C
        # zero-filled by hipMemset; ``uncached`` (flag words): fine-grained memory no GPU caches
        self.h = C.SymmetricBuffer(self.nbytes, ctx.device_index, bool(uncached))
        handles: List = [None] * ctx.world
        mine = bytes(self.h.ipc_handle())
        if ctx.world > 1:
            dist.all_gather_object(handles, mine)
        else:
            handles = [mine]
        self.h.open_peers(handles, ctx.rank)
        self.tensor = torch.from_dlpack(C.buffer_dlpack(self.h, ctx.device_index))

    def ptr(self, owner: Optional[int] = None) -> int:
        return self.h.local() if owner is None or owner == self.ctx.rank else self.h.peer(owner)

    def close_peers(self) -> None:
        if self.h is not None:
            self.h.close_peers()

    def release(self) -> None:
        """Free now. Every rank must have closed its mapping first (see BoundPlan.close)."""
        self.tensor = None
        if self.h is not None:
            self.h.release()
            self.h = None

    def close(self) -> None:
        self.close_peers()
        self.release()


def check_single_node(world: int) -> None:
    """HIP IPC symmetric memory (every ``backend=ipc`` plan) maps peers' HBM over xGMI, which
    only exists between GPUs of one node: refuse a multi-node job with a clear message instead
    of failing inside hipIpcOpenMemHandle. Hostnames are compared over the control group (no
    reliance on launcher-specific local-size variables)."""
    import socket

    import torch.distributed as dist

    if world <= 1:
        return
    names: List = [None] * world
    dist.all_gather_object(names, socket.gethostname())
    hosts = sorted(set(names))
    if len(hosts) > 1:
        raise RuntimeError(
            f"backend=ipc needs every rank on one node (HIP IPC over xGMI); this job spans "
            f"{len(hosts)} hosts ({', '.join(hosts[:4])}{', ...' if len(hosts) > 4 else ''}): "
            "use backend=rccl")


class NativeContext:
    def __init__(self, communicator):
        from ddlb_amd.ops import load

        if not communicator.is_gpu:
            raise RuntimeError("the native data plane needs a ROCm GPU")
        self.C = load()
        if os.environ.get("DDLB_CRASH_BT", "0") == "1":
            self.C.install_crash_handler()  # native frames on SIGSEGV / SIGABRT (diagnostics)
        self.comm = communicator
        self.rank = communicator.rank
        self.world = communicator.world_size
        self.device_index = communicator.device.index
        self._rccl: Dict[int, object] = {}   # CTA cap (0 = RCCL's default) -> communicator
        self._owned: List = []
        self._single_node_checked = False

    def rccl(self, max_ctas: int = 0):
        """Our own RCCL communicator (lazily created, collective over all ranks). ``max_ctas`` > 0:
        a communicator whose kernels launch at most that many workgroups (``ncclConfig_t``
        maxCTAs), the one a plan with an RCCL-fed flag-gated GEMM binds (see
        :func:`rccl_gate_cap`); one communicator per cap, created in bind order (identical on
        every rank)."""
        import torch.distributed as dist

        cap = max(int(max_ctas), 0)
        if cap not in self._rccl:
            obj = [bytes(self.C.RcclComm.unique_id()) if self.rank == 0 else None]
            if self.world > 1:
                dist.broadcast_object_list(obj, src=0)
            comm = self.C.RcclComm(obj[0], self.world, self.rank, self.device_index, cap)
            # (comm.max_ctas is the cap WE passed in ncclConfig_t, a binding consistency check
            # only; what RCCL actually needs beside a gated GEMM is observed by the rccl_cap
            # preflight phase, which holds num_cus - cap CUs while the capped collective runs)
            if int(comm.max_ctas) != cap:
                raise RuntimeError(f"RCCL communicator binding: asked for a {cap}-CTA cap, "
                                   f"recorded {comm.max_ctas}")
            self._rccl[cap] = comm
        return self._rccl[cap]

    def symmetric(self, nbytes: int, uncached: bool = False) -> SymmetricBuffer:
        if not self._single_node_checked:
            check_single_node(self.world)
            self._single_node_checked = True
        buf = SymmetricBuffer(self, nbytes, uncached=uncached)
        self._owned.append(buf)
        return buf

    def release_symmetric(self, bufs) -> None:
        """Collective teardown: unmap peers everywhere, barrier, then free locally."""
        import torch

        torch.cuda.synchronize()
        for b in bufs:
            b.close_peers()
        if self.world > 1:
            self.comm.barrier()
        for b in bufs:
            b.release()
        self._owned = [b for b in self._owned if b.h is not None]

    def bind(self, plan: Plan, externals=None, trace: bool = False) -> "BoundPlan":
        return BoundPlan(self, plan, externals, trace=trace)

    def close(self) -> None:
        for b in self._owned:
            b.close()
        self._owned = []
        comms, self._rccl = list(self._rccl.values()), {}
        first = None
        for c in comms:  # every communicator is destroyed even if one destroy() raises
            try:
                c.destroy()
            except Exception as e:  # noqa: BLE001 (re-raised below)
                first = first or e
        if first is not None:
            raise first


def rccl_buffers(plan: Plan) -> List[str]:
    """Names of the buffers the plan's RCCL ops read or write (registration candidates)."""
    names: List[str] = []
    for op in plan.ops:
        if op.kind in RCCL_OPS:
            for key in ("send", "recv", "buf"):
                ref = op.args.get(key)
                if ref is not None and ref.buf not in names:
                    names.append(ref.buf)
    return names


def rccl_gate_cap(plan: Plan) -> int:
    """CTA cap of the RCCL communicator a plan must bind (0 = RCCL's default).

    A plan whose flag-gated GEMM is fed by RCCL collectives (the RCCL-fed fused pipelines) is
    deadlock-free only if the collectives can always be resident beside the spinning tiles. The
    gated persistent GEMM takes ``num_cus - reserve_cus`` CUs (one workgroup each, a whole CU's
    register file), so the builder records ``rccl_max_ctas`` <= ``reserve_cus`` in the plan and the
    communicator is created with that cap (``ncclConfig_t`` maxCTAs): GEMM grid + RCCL grid <=
    num_cus holds by construction, whatever RCCL's default channel count is on the node. A CU split
    (``comm_cus`` > 0: the collectives on CUs of their own) needs no cap. Anything else is refused
    here, before a launch could hang."""
    gated = [op for op in plan.ops if op.kind == OP_GEMM and op.args.get("flags") is not None
             and op.stream == 0]
    if not gated or not any(op.kind in RCCL_OPS for op in plan.ops):
        return int(plan.meta.get("rccl_max_ctas", 0))
    cap = int(plan.meta.get("rccl_max_ctas", 0))
    if int(plan.meta.get("comm_cus", 0)) > 0:
        return cap
    reserve = min(int(op.args.get("reserve_cus", 0)) for op in gated)
    if cap <= 0 or cap > reserve:
        raise ValueError(f"RCCL-fed flag-gated GEMM: the communicator's CTA cap ({cap}) must be "
                         f"in [1, reserve_cus = {reserve}] (or use comm_cus > 0), else a collective "
                         "may not fit beside the spinning tiles")
    return cap


class BoundPlan:
    """``externals`` maps a LOCAL buffer name to an existing device tensor that backs it
    (zero-copy chaining: e.g. the columnwise output feeding the rowwise input of an MLP).

    Plan settings applied here (``plan.meta``): ``register`` — the buffers RCCL touches come from
    ``ncclMemAlloc`` and are registered with our communicator (``ncclCommRegister``);
    ``comm_cus`` — the executor's CU split (side streams on that many CUs, stream-0 ops on the
    rest). ``trace`` (or ``DDLB_PLAN_TRACE=1``) turns on a roctx range per op."""

    def __init__(self, ctx: NativeContext, plan: Plan, externals=None, trace: bool = False):
        import torch

        self.ctx, self.plan = ctx, plan
        self.local: Dict[str, torch.Tensor] = {}
        self.sym: Dict[str, SymmetricBuffer] = {}
        self.rmem: Dict[str, object] = {}
        self._uncached: List = []
        dev = torch.device("cuda", ctx.device_index)
        externals = dict(externals or {})
        registered = set(rccl_buffers(plan)) if plan.meta.get("register") else set()
        # an RCCL-fed flag-gated GEMM binds a CTA-capped communicator (checked, CPU-testable)
        self.rccl_cap = rccl_gate_cap(plan)
        for name, spec in plan.buffers.items():  # dict order == identical on every rank
            if name in registered and name not in externals and not spec.symmetric:
                # zero-copy RCCL buffer: ncclMemAlloc + ncclCommRegister on our communicator
                mem = ctx.C.RcclMem(ctx.rccl(self.rccl_cap), max(spec.nbytes, 16),
                                    ctx.device_index)
                self.rmem[name] = mem
                self.local[name] = torch.from_dlpack(ctx.C.rccl_mem_dlpack(mem, ctx.device_index))
                continue
            if name in externals:
                t = externals.pop(name)
                if spec.symmetric:
                    raise ValueError(f"buffer {name} is symmetric; it cannot be external")
                if not t.is_contiguous() or t.device != dev:
                    raise ValueError(f"external {name} must be a contiguous tensor on {dev}")
                raw = t.view(-1).view(torch.uint8)
                if raw.numel() < spec.nbytes:
                    raise ValueError(f"external {name}: {raw.numel()} B < {spec.nbytes} B needed")
                self.local[name] = raw
            elif spec.symmetric:
                # zero-initialised symmetric buffers are the cross-process flag words: peers
                # write them over xGMI while this GPU polls, so they live in uncached memory
                self.sym[name] = ctx.symmetric(spec.nbytes, uncached=spec.zero)
            elif spec.zero:
                # local flag words (e.g. the ARRIVE flags an RCCL-fed gated GEMM polls, set by
                # signal kernels on another stream): uncached too, so a tile polling from one
                # XCD never spins on a stale line of its L2 while the store sits in another's
                # (r4 budget: erratic 0.18-0.69 ms plan times with cached flags)
                h = ctx.C.SymmetricBuffer(max(spec.nbytes, 16), ctx.device_index, True)
                self._uncached.append(h)
                self.local[name] = torch.from_dlpack(ctx.C.buffer_dlpack(h, ctx.device_index))
            else:
                self.local[name] = torch.zeros(max(spec.nbytes, 16), dtype=torch.uint8,
                                               device=dev)
        if externals:
            raise ValueError(f"externals {sorted(externals)} are not buffers of this plan")
        for name, spec in plan.buffers.items():
            if spec.table is not None:
                addrs = torch.tensor([self.resolve(r) for r in spec.table], dtype=torch.int64)
                self.local[name][:8 * len(spec.table)].copy_(addrs.view(torch.uint8))
        words = plan.encode(self.resolve)
        C = ctx.C
        self.ex = C.PlanExecutor(ctx.device_index, plan.nstreams, max(plan.nevents, 1),
                                 list(plan.stream_priority))
        self.ex.load(words)
        if any(op.kind in RCCL_OPS for op in plan.ops):
            self.ex.set_comm(ctx.rccl(self.rccl_cap))
            if any(op.kind == OP_GEMM and op.args.get("flags") is not None for op in plan.ops):
                self._warm_rccl()
        if plan.meta.get("comm_cus", 0):
            self.ex.set_cu_split(int(plan.meta["comm_cus"]))
        if trace or os.environ.get("DDLB_PLAN_TRACE", "0") == "1":
            self.ex.set_trace(True, plan.labels())
        torch.cuda.synchronize(dev)

    def _warm_rccl(self) -> None:
        """Run the plan's RCCL calls once, alone, before its first real run: RCCL sets up its
        peer connections lazily inside the first collective of each kind, and a flag-gated GEMM
        enqueued ahead of the collectives (the RCCL-fed fused pipelines) must never be on the
        device while that setup runs (any device-wide synchronisation in it would wait for the
        spinning tiles). Every rank binds the same plan, so every rank issues the same calls."""
        import torch

        from ddlb_amd.parallel.plan import OP_GROUP_END, OP_GROUP_START

        warm = Plan(self.plan.rank, self.plan.world, nstreams=self.plan.nstreams,
                    stream_priority=list(self.plan.stream_priority))
        warm.ops = [op for op in self.plan.ops
                    if op.kind in RCCL_OPS or op.kind in (OP_GROUP_START, OP_GROUP_END)]
        ex = self.ctx.C.PlanExecutor(self.ctx.device_index, warm.nstreams, 1,
                                     list(warm.stream_priority))
        ex.load(warm.encode(self.resolve))
        ex.set_comm(self.ctx.rccl(self.rccl_cap))
        ex.run(_raw_stream(self.ctx.device_index))
        torch.cuda.synchronize()
        del ex

    def resolve(self, ref: Ref) -> int:
        if ref.buf in self.sym:
            base = self.sym[ref.buf].ptr(ref.owner)
            size = self.sym[ref.buf].nbytes
        else:
            if ref.owner is not None and ref.owner != self.ctx.rank:
                raise ValueError(f"buffer {ref.buf} is local; cannot address rank {ref.owner}")
            base = self.local[ref.buf].data_ptr()
            size = self.local[ref.buf].numel()
        if not 0 <= ref.off <= size:
            raise ValueError(f"ref {ref} outside buffer of {size} bytes")
        return base + ref.off

    def buffer(self, name: str):
        return self.sym[name].tensor if name in self.sym else self.local[name]

    def view(self, loc):
        """Typed ``[rows, cols]`` tensor view of a :class:`TensorLoc`."""
        raw = self.buffer(loc.buf)
        n = loc.rows * loc.cols * DT_SIZE[loc.dtype]
        return raw[loc.off:loc.off + n].view(TORCH_DT[loc.dtype]).view(loc.rows, loc.cols)

    def enable_graph(self, on: bool = True) -> None:
        """Replay the whole plan from one captured hipGraph: one launch per run instead of one
        HIP / RCCL call per op (signal plans read a device-side run counter in this mode)."""
        if on and not graph_replay_supported():
            raise RuntimeError(
                "hipGraph replay needs at least 4 hardware queues per process: with "
                f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')} the HIP runtime of this "
                "image crashes in hipGraphLaunch (profiles/r02/r2_17_*)")
        if os.environ.get("DDLB_CRASH_BT", "0") == "1":
            self.ctx.C.install_crash_handler()  # (re)install right before the capture
        self.ex.enable_graph(on)

    def run(self, stream: Optional[int] = None) -> int:
        if stream is None:
            stream = _raw_stream(self.ctx.device_index)
        return self.ex.run(stream)

    def set_timeline(self, on: bool = True) -> None:
        """Record per-op GPU timing events on the next runs (see :meth:`timeline`)."""
        self.ex.set_timeline(bool(on))

    def timeline(self) -> List[Dict]:
        """Per-op timing of the LAST run: ``start_ms`` / ``end_ms`` from the fork on the
        caller's stream. An op's end is measured (an event on its stream right after it); its
        start is the end of the previous op on the same stream, so waits show up as the time an
        op spent blocked behind its dependencies."""
        ends = self.ex.timeline()
        host = self.ex.host_times()
        last: Dict[int, float] = {}
        rows = []
        for i, (op, end) in enumerate(zip(self.plan.ops, ends)):
            start = last.get(op.stream, 0.0)
            end = max(float(end), start)
            last[op.stream] = end
            rows.append({"index": i, "op": op.name, "stream": op.stream, "start_ms": start,
                         "end_ms": end, "host_us": float(host[i]) if i < len(host) else 0.0})
        return rows

    def check_health(self) -> None:
        code = self.ex.read_timeout()
        if code:
            raise RuntimeError(f"native plan: a bounded spin gave up (code {code}); a peer did not "
                               "signal in time")

    def close(self) -> None:
        import torch

        torch.cuda.synchronize()
        self.ex = None
        self.ctx.release_symmetric(list(self.sym.values()))
        for name in list(self.rmem):
            # deregister while the communicator lives; ncclMemFree happens when the last view
            # goes (a rowwise OUT returned by run() stays readable after close)
            self.local.pop(name, None)
            self.rmem.pop(name).release()
        self.sym, self.local = {}, {}
        for h in self._uncached:  # local uncached flag words: no peer maps them
            h.release()
        self._uncached = []
