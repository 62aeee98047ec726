"""Plan IR: the host-side schedule of a distributed-GEMM algorithm.

The reference expresses its pipelines as nvFuser fusions that the MultiDeviceExecutor lowers to a
host IR of per-stream collectives + matmuls (``ddlb/primitives/TPColumnwise/fuser.py:59-146``,
``TPRowwise/fuser.py:62-169``). Here an algorithm is a Python function that emits a :class:`Plan`:
a flat op list over **named buffers** and a fixed set of HIP streams. The same plan is

* encoded to int64 words and executed by the native C++ ``PlanExecutor`` (one call per run), and
* interpreted by :mod:`ddlb_amd.parallel.sim` on the CPU (d simulated ranks, byte-exact
  buffers) with a happens-before race checker — the test bed for the layout math when no
  multi-GPU node is at hand.

Pointers are symbolic :class:`Ref` ``(buffer, byte offset, owner rank)``; ``owner=None`` means the
local copy, an integer means that peer's copy of a *symmetric* buffer (IPC-mapped).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

OP_WORDS = 34
(OP_NOP, OP_GEMM, OP_RECORD, OP_WAIT, OP_ALLGATHER, OP_REDUCE_SCATTER, OP_SEND, OP_RECV,
 OP_GROUP_START, OP_GROUP_END, OP_COPY, OP_SIGNAL, OP_WAIT_SIGNAL, OP_REDUCE, OP_MEMSET,
 OP_COPY_MULTI, OP_COPY_BATCH) = range(17)
OP_NAMES = {OP_NOP: "nop", OP_GEMM: "gemm", OP_RECORD: "record", OP_WAIT: "wait",
            OP_ALLGATHER: "allgather", OP_REDUCE_SCATTER: "reduce_scatter", OP_SEND: "send",
            OP_RECV: "recv", OP_GROUP_START: "group_start", OP_GROUP_END: "group_end",
            OP_COPY: "copy", OP_SIGNAL: "signal", OP_WAIT_SIGNAL: "wait_signal",
            OP_REDUCE: "reduce", OP_MEMSET: "memset", OP_COPY_MULTI: "copy_multi",
            OP_COPY_BATCH: "copy_batch"}
RCCL_OPS = (OP_ALLGATHER, OP_REDUCE_SCATTER, OP_SEND, OP_RECV)

# dtype codes (csrc/gemm/gemm.h)
DT_F32, DT_F16, DT_BF16, DT_FP8, DT_F64, DT_U8 = 0, 1, 2, 3, 4, 5
DT_SIZE = {DT_F32: 4, DT_F16: 2, DT_BF16: 2, DT_FP8: 1, DT_F64: 8, DT_U8: 1}
DT_NAME = {DT_F32: "float32", DT_F16: "float16", DT_BF16: "bfloat16", DT_FP8: "float8_e4m3fn",
           DT_F64: "float64", DT_U8: "uint8"}
NAME_DT = {v: k for k, v in DT_NAME.items()}

# fused GEMM epilogue activations (csrc/gemm/gemm.h ACT_*)
ACT_NONE, ACT_GELU, ACT_RELU, ACT_SILU = 0, 1, 2, 3
ACT_CODE = {"none": ACT_NONE, "gelu": ACT_GELU, "relu": ACT_RELU, "silu": ACT_SILU}

# copy / signal methods
COPY_ENGINE, COPY_KERNEL = 0, 1
SIG_KERNEL, SIG_STREAM = 0, 1
# a wait the preceding in-kernel all-gather launch already performs (its copy role waits for the
# ACKs before the launch ends): skipped by the executor, simulated as an ordinary wait
SIG_IN_LAUNCH = 2


@dataclass(frozen=True)
class Ref:
    buf: str
    off: int = 0          # bytes
    owner: Optional[int] = None  # None = local; rank = that rank's copy (symmetric buffers)

    def __add__(self, nbytes: int) -> "Ref":
        return Ref(self.buf, self.off + int(nbytes), self.owner)

    def at(self, owner: Optional[int]) -> "Ref":
        return Ref(self.buf, self.off, owner)


@dataclass
class BufferSpec:
    name: str
    nbytes: int
    symmetric: bool = False
    zero: bool = False          # must start zeroed (flags)
    table: Optional[List[Ref]] = None  # pointer table: filled with the refs' addresses at bind


@dataclass
class Op:
    kind: int
    stream: int
    args: Dict = field(default_factory=dict)

    @property
    def name(self) -> str:
        return OP_NAMES[self.kind]


class Plan:
    """Op list + buffer declarations for ONE rank."""

    def __init__(self, rank: int, world: int, nstreams: int = 1,
                 stream_priority: Optional[Sequence[int]] = None):
        self.rank, self.world = rank, world
        self.nstreams = nstreams
        self.stream_priority = list(stream_priority or [0] * nstreams)
        self.ops: List[Op] = []
        self.buffers: Dict[str, BufferSpec] = {}
        self.nevents = 0
        self.meta: Dict = {}

    # ------------------------------------------------------------------ declarations
    def buffer(self, name: str, nbytes: int, symmetric: bool = False, zero: bool = False) -> Ref:
        nbytes = int(nbytes)
        if name in self.buffers:
            b = self.buffers[name]
            if b.nbytes != nbytes or b.symmetric != symmetric:
                raise ValueError(f"buffer {name} redeclared differently")
        else:
            self.buffers[name] = BufferSpec(name, nbytes, symmetric, zero)
        return Ref(name, 0, None)

    def event(self) -> int:
        self.nevents += 1
        return self.nevents - 1

    def _add(self, kind, stream, **args) -> Op:
        if not 0 <= stream < self.nstreams:
            raise ValueError(f"stream {stream} out of range (nstreams={self.nstreams})")
        op = Op(kind, stream, args)
        self.ops.append(op)
        return op

    # ------------------------------------------------------------------ ops
    def gemm(self, stream: int, a: Ref, b: Ref, c: Ref, *, M: int, N: int, K: int, lda: int,
             ldb: int, ldc: int, din: int, dout: int, a_grp: int = 0, a_gstride: int = 0,
             c_grp: int = 0, c_gstride: int = 0, tile: int = 0, mode: int = 0,
             flags: Optional[Ref] = None, flag_rows: int = 0, nshards: int = 1,
             first_shard: int = 0, tile_order: int = 0, act: int = 0,
             a_shards: Optional[Sequence[Ref]] = None, shard_rows: int = 0,
             nsub: int = 1, reserve_cus: int = 0, ag: Optional[dict] = None,
             c_shards: Optional[Sequence[Ref]] = None, c_shard_rows: int = 0,
             ksplit: int = 1) -> Op:
        """``a_shards``: A row block s (``shard_rows`` rows each) is read from ``a_shards[s]``
        (a peer's copy for a direct-access GEMM that pulls its operand over xGMI).
        ``flags`` (arrival-gated tiles): shard ``i`` = rows ``[i*flag_rows, (i+1)*flag_rows)`` may
        be read once ``flags[i]`` reaches the run's epoch; with ``tile_order`` the tiles are
        dispatched shard by shard from ``first_shard`` — ``nsub`` > 1 splits each producer's
        shard into that many row blocks (shard = producer * nsub + block) dispatched block-major
        (block 0 of every producer first), the order chunked pulls land in. A persistent
        flag-gated GEMM leaves ``reserve_cus`` CUs free for the kernels that set the flags.
        ``ag`` = in-kernel all-gather (``dict(ctas, parts, rank, src, ack, ready, count)``, see
        csrc/gemm/gemm.h ``ag_ctas``): the launch's first ``ctas`` workgroups pull row block b of
        every producer p (``src[p]``, same rows) into A, set ``flags[p * nsub + b]`` and ACK p
        (``ack[p]``) after READY (``ready[p]``); the GEMM tiles gate on those flags.
        ``c_shards`` (direct-store C): C row block s (``c_shard_rows`` rows) is written at
        ``c_shards[s]`` — e.g. the peers' receive slots, so the epilogue stores a reduce-scatter's
        partials straight over xGMI; ``tile_order=2`` interleaves the blocks (every destination's
        tiles in flight at once). ``ksplit`` > 1: K-split, ``K`` is the slice length (``lda`` /
        ``ldb`` the full rows); slice s reads A / B columns ``[s K, (s + 1) K)`` and writes its
        partial product at ``c + s * M * ldc`` elements (plain rows only; the caller sums them
        with a reduce op)."""
        if ksplit < 1 or (ksplit > 1 and (flags is not None or a_shards is not None or
                                          c_shards is not None or ag is not None or act or
                                          a_grp not in (0, M) or c_grp not in (0, M))):
            raise ValueError("ksplit > 1 takes plain rows only (no flags, tables, all-gather, "
                             "activation or grouped rows)")
        if nsub < 1 or nshards % nsub:
            raise ValueError(f"nsub ({nsub}) must divide nshards ({nshards})")
        if ag is not None:
            npro = nshards // nsub
            if flags is None or len(ag["src"]) != npro or len(ag["ack"]) != npro:
                raise ValueError("in-kernel all-gather needs flags and one src / ack per producer")
            if not 1 <= ag["ctas"] < 1 << 20 or not 1 <= ag["parts"] < 1 << 20:
                raise ValueError("ag ctas / parts out of range")
            if not 0 <= ag.get("mode", 0) < 32:
                raise ValueError("ag mode out of range (csrc/gemm/gemm.h AgMode bits)")
            acks_in = list(ag.get("wait_acks") or [])
            if bool(acks_in) != bool(ag.get("mode", 0) & 16) or (acks_in and len(acks_in) != npro):
                raise ValueError("ag mode 16 (AG_WAIT_ACKS) needs wait_acks: one local ACK word "
                                 "per producer (and only then)")
            ag = dict(ag, table=self.table(f"__agtab{len(self.buffers)}",
                                           list(ag["src"]) + list(ag["ack"]) +
                                           [ag["ready"], ag["count"]] + acks_in))
        c_table = None
        if c_shards is not None:
            if c_shard_rows <= 0 or len(c_shards) * c_shard_rows < M or c_grp not in (0, M):
                raise ValueError("c_shards must cover the M rows (no grouped C rows)")
            c_table = self.table(f"__ctab{len(self.buffers)}", c_shards)
        if tile_order == 2 and (nshards < 1 or M % nshards):
            raise ValueError("tile_order=2 needs nshards dividing M")
        a_table = None
        if a_shards is not None:
            if shard_rows <= 0 or len(a_shards) * shard_rows < M:
                raise ValueError("a_shards must cover the M rows")
            a_table = self.table(f"__atab{len(self.buffers)}", a_shards)
        return self._add(OP_GEMM, stream, a=a, b=b, c=c, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=ldc,
                         din=din, dout=dout, a_grp=a_grp, a_gstride=a_gstride, c_grp=c_grp,
                         c_gstride=c_gstride, tile=tile, mode=mode, flags=flags,
                         flag_rows=flag_rows, nshards=nshards, first_shard=first_shard,
                         tile_order=tile_order, act=act,
                         a_shards=list(a_shards) if a_shards is not None else None,
                         shard_rows=shard_rows, a_table=a_table, nsub=nsub,
                         reserve_cus=reserve_cus, ag=ag,
                         c_shards=list(c_shards) if c_shards is not None else None,
                         c_shard_rows=c_shard_rows, c_table=c_table, ksplit=ksplit)

    def table(self, name: str, refs: Sequence[Ref]) -> Ref:
        """Device array of 64-bit addresses of ``refs`` (written once when the plan is bound)."""
        self.buffers[name] = BufferSpec(name, max(16, 8 * len(refs)), table=list(refs))
        return Ref(name, 0, None)

    def record(self, stream: int, event: int) -> Op:
        return self._add(OP_RECORD, stream, event=event)

    def wait(self, stream: int, event: int) -> Op:
        return self._add(OP_WAIT, stream, event=event)

    def edge(self, src_stream: int, dst_stream: int) -> None:
        """Make everything queued so far on ``src_stream`` precede later ops of ``dst_stream``."""
        if src_stream == dst_stream:
            return
        e = self.event()
        self.record(src_stream, e)
        self.wait(dst_stream, e)

    def allgather(self, stream: int, send: Ref, recv: Ref, count: int, dtype: int) -> Op:
        return self._add(OP_ALLGATHER, stream, send=send, recv=recv, count=count, dtype=dtype)

    def reduce_scatter(self, stream: int, send: Ref, recv: Ref, count: int, dtype: int) -> Op:
        return self._add(OP_REDUCE_SCATTER, stream, send=send, recv=recv, count=count, dtype=dtype)

    def send(self, stream: int, buf: Ref, count: int, dtype: int, peer: int) -> Op:
        return self._add(OP_SEND, stream, buf=buf, count=count, dtype=dtype, peer=peer)

    def recv(self, stream: int, buf: Ref, count: int, dtype: int, peer: int) -> Op:
        return self._add(OP_RECV, stream, buf=buf, count=count, dtype=dtype, peer=peer)

    def group_start(self, stream: int) -> Op:
        return self._add(OP_GROUP_START, stream)

    def group_end(self, stream: int) -> Op:
        return self._add(OP_GROUP_END, stream)

    def copy(self, stream: int, dst: Ref, src: Ref, nbytes: int, method: int = COPY_ENGINE,
             max_blocks: int = 0) -> Op:
        return self._add(OP_COPY, stream, dst=dst, src=src, nbytes=int(nbytes), method=method,
                         max_blocks=max_blocks)

    def copy_multi(self, stream: int, segs: Sequence[Tuple[Ref, Ref, int]],
                   max_blocks: int = 0) -> Op:
        if not 1 <= len(segs) <= 8:
            raise ValueError("copy_multi takes 1..8 segments")
        return self._add(OP_COPY_MULTI, stream, segs=list(segs), max_blocks=max_blocks)

    def copy_batch(self, stream: int, segs: Sequence[Tuple[Ref, Ref, int]]) -> Op:
        """Copy-engine copies submitted together (``hipMemcpyBatchAsync``: the
        ``batch_memcpy`` protocol, one API call per block across all peers)."""
        if not 1 <= len(segs) <= 8:
            raise ValueError("copy_batch takes 1..8 segments")
        return self._add(OP_COPY_BATCH, stream, segs=list(segs))

    def signal(self, stream: int, flags: Sequence[Ref], method: int = SIG_STREAM,
               delta: int = 0) -> Op:
        if not 1 <= len(flags) <= 16:
            raise ValueError("signal takes 1..16 flags")
        return self._add(OP_SIGNAL, stream, flags=list(flags), method=method, delta=delta)

    def wait_signal(self, stream: int, flags: Sequence[Ref], method: int = SIG_STREAM,
                    delta: int = 0) -> Op:
        if not 1 <= len(flags) <= 16:
            raise ValueError("wait_signal takes 1..16 flags")
        return self._add(OP_WAIT_SIGNAL, stream, flags=list(flags), method=method, delta=delta)

    def reduce(self, stream: int, dst: Ref, srcs: Sequence[Ref], count: int, dtype: int) -> Op:
        if not 1 <= len(srcs) <= 16:
            raise ValueError("reduce takes 1..16 sources")
        return self._add(OP_REDUCE, stream, dst=dst, srcs=list(srcs), count=count, dtype=dtype)

    def memset(self, stream: int, dst: Ref, nbytes: int, value: int = 0) -> Op:
        return self._add(OP_MEMSET, stream, dst=dst, nbytes=nbytes, value=value)

    # ------------------------------------------------------------------ encoding
    def encode(self, resolve: Callable[[Ref], int]) -> List[int]:
        """Flatten to ``OP_WORDS`` int64 per op; ``resolve`` maps a Ref to a device address."""
        words: List[int] = []
        for op in self.ops:
            w = [0] * OP_WORDS
            w[0], w[1] = op.kind, op.stream
            a = op.args
            k = op.kind
            if k == OP_GEMM:
                w[2:12] = [resolve(a["a"]), resolve(a["b"]), resolve(a["c"]), a["lda"], a["ldb"],
                           a["ldc"], a["a_grp"], a["a_gstride"], a["c_grp"], a["c_gstride"]]
                w[12:19] = [a["M"], a["N"], a["K"], a["din"], a["dout"], a["tile"], a["mode"]]
                w[19] = resolve(a["flags"]) if a["flags"] is not None else 0
                w[20:25] = [a["flag_rows"], a["nshards"], a["first_shard"], a["tile_order"],
                            a.get("act", 0)]
                if a.get("a_table") is not None:
                    w[25], w[26] = resolve(a["a_table"]), a["shard_rows"]
                w[27], w[28] = a.get("nsub", 1), a.get("reserve_cus", 0)
                g = a.get("ag")
                if g is not None:
                    w[29] = (g["ctas"] | (g["parts"] << 20) | (g["rank"] << 40) |
                             (g.get("mode", 0) << 56))
                    w[30] = resolve(g["table"])
                if a.get("c_table") is not None:
                    w[32], w[33] = resolve(a["c_table"]), a["c_shard_rows"]
                w[31] = a.get("ksplit", 1)
            elif k in (OP_RECORD, OP_WAIT):
                w[2] = a["event"]
            elif k in (OP_ALLGATHER, OP_REDUCE_SCATTER):
                w[2:6] = [resolve(a["send"]), resolve(a["recv"]), a["count"], a["dtype"]]
            elif k in (OP_SEND, OP_RECV):
                w[2:6] = [resolve(a["buf"]), a["count"], a["dtype"], a["peer"]]
            elif k == OP_COPY:
                w[2:7] = [resolve(a["dst"]), resolve(a["src"]), a["nbytes"], a["method"],
                          a["max_blocks"]]
            elif k in (OP_COPY_MULTI, OP_COPY_BATCH):
                w[2], w[3] = len(a["segs"]), a.get("max_blocks", 0)
                for i, (d, s, n) in enumerate(a["segs"]):
                    w[4 + 3 * i:7 + 3 * i] = [resolve(d), resolve(s), n]
            elif k in (OP_SIGNAL, OP_WAIT_SIGNAL):
                w[2], w[3], w[4] = len(a["flags"]), a["method"], a["delta"]
                for i, f in enumerate(a["flags"]):
                    w[5 + i] = resolve(f)
            elif k == OP_REDUCE:
                w[2:6] = [resolve(a["dst"]), a["count"], a["dtype"], len(a["srcs"])]
                for i, s in enumerate(a["srcs"]):
                    w[6 + i] = resolve(s)
            elif k == OP_MEMSET:
                w[2:5] = [resolve(a["dst"]), a["nbytes"], a["value"]]
            words.extend(int(x) for x in w)
        return words

    def labels(self) -> List[str]:
        """One trace label per op (the roctx range names of ``PlanExecutor.set_trace``): GEMMs
        numbered in issue order ("gemm s3"; "+ag" in-kernel all-gather, "+gated" arrival
        flags), copies by peer and block ("copy p2 b1"), collectives numbered, flag ops by
        their first flag word."""
        out: List[str] = []
        count: Dict[str, int] = {}
        blocks: Dict[Tuple[str, int], int] = {}

        def nxt(key: str) -> int:
            count[key] = count.get(key, 0) + 1
            return count[key] - 1

        def peer_of(refs) -> int:
            for r in refs:
                if r.owner is not None and r.owner != self.rank:
                    return r.owner
            return self.rank

        for op in self.ops:
            a, k = op.args, op.kind
            if k == OP_GEMM:
                tag = "+ag" if a.get("ag") else ("+gated" if a.get("flags") is not None else "")
                out.append(f"gemm s{nxt('gemm')}{tag}")
            elif k in (OP_COPY, OP_COPY_MULTI, OP_COPY_BATCH):
                refs = ([a["src"], a["dst"]] if k == OP_COPY else
                        [r for seg in a["segs"] for r in seg[:2]])
                p = peer_of(refs)
                key = ("copy", p)
                blocks[key] = blocks.get(key, -1) + 1
                multi = "" if k == OP_COPY else f" x{len(a['segs'])}"
                out.append(f"{OP_NAMES[k]} p{p} b{blocks[key]}{multi}")
            elif k in (OP_SIGNAL, OP_WAIT_SIGNAL):
                f = a["flags"][0]
                out.append(f"{OP_NAMES[k]} {f.buf}+{f.off}" +
                           (f"@{f.owner}" if f.owner is not None else "") +
                           (f" x{len(a['flags'])}" if len(a["flags"]) > 1 else ""))
            elif k in RCCL_OPS:
                out.append(f"{OP_NAMES[k]} #{nxt(OP_NAMES[k])}")
            else:
                out.append(OP_NAMES[k])
        return out

    def describe(self) -> str:
        """Human-readable listing (``python -m ddlb_amd.parallel.explain`` prints this)."""
        lines = [f"plan rank={self.rank}/{self.world} streams={self.nstreams} "
                 f"events={self.nevents} ops={len(self.ops)}"]
        for name, b in self.buffers.items():
            lines.append(f"  buffer {name}: {b.nbytes} B{' symmetric' if b.symmetric else ''}")
        for i, op in enumerate(self.ops):
            parts = []
            for key, v in op.args.items():
                if isinstance(v, Ref):
                    v = f"{v.buf}+{v.off}" + (f"@{v.owner}" if v.owner is not None else "")
                elif isinstance(v, list) and v and isinstance(v[0], Ref):
                    v = "[" + ",".join(f"{x.buf}+{x.off}" + (f"@{x.owner}" if x.owner is not None
                                                             else "") for x in v) + "]"
                parts.append(f"{key}={v}")
            lines.append(f"  {i:3d} s{op.stream} {op.name:14s} " + " ".join(parts))
        return "\n".join(lines)
