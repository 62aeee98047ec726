"""CPU simulator + race/deadlock checker for plans (no GPU needed).

Executes the plans of ``d`` simulated ranks with the semantics the native executor relies on:

* each rank runs epochs one after another (the executor forks every stream from the caller's
  stream and joins them back, so nothing of epoch e+1 starts before epoch e finished);
* inside an epoch, streams are independent FIFO queues; an op may start when it is at the head
  of its stream and its dependencies are met: ``wait`` -> the matching ``record`` ran;
  ``wait_signal`` -> every flag >= epoch + delta; collectives / send-recv groups -> every rank
  reached the same collective (matched by issue order, as RCCL requires);
* data is real: every buffer is a byte tensor per rank, GEMMs / reductions run in f32 and round
  to the output dtype, collectives move bytes exactly as RCCL would.

If no op can make progress before all finished, the plan **deadlocks** -> :class:`Deadlock`.
With ``check_races=True`` every op carries a vector clock over (rank, stream); two accesses to
overlapping bytes of the same physical buffer, at least one a write, that are not ordered by
happens-before raise :class:`RaceDetected` (flag words are synchronisation and excluded).

This is the test bed for the layout math and the synchronisation protocol of every algorithm
(SURVEY.md §7.4 "Layout tests on CPU", §5.2 race detection).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ddlb_amd.parallel.plan import (DT_BF16, DT_F16, DT_F32, DT_F64, DT_FP8, DT_SIZE, DT_U8,
                                    OP_ALLGATHER, OP_COPY, OP_COPY_BATCH, OP_COPY_MULTI, OP_GEMM,
                                    OP_GROUP_END,
                                    OP_GROUP_START, OP_MEMSET, OP_NAMES, OP_NOP, OP_RECORD, OP_RECV,
                                    OP_REDUCE, OP_REDUCE_SCATTER, OP_SEND, OP_SIGNAL, OP_WAIT,
                                    OP_WAIT_SIGNAL, Plan, Ref)

TORCH_DT = {DT_F32: torch.float32, DT_F16: torch.float16, DT_BF16: torch.bfloat16,
            DT_FP8: torch.float8_e4m3fn, DT_F64: torch.float64, DT_U8: torch.uint8}


def apply_act(x: torch.Tensor, act: int) -> torch.Tensor:
    """f32 reference of the fused GEMM epilogue activations (csrc/gemm/gemm_mfma.hip act1)."""
    if act == 1:
        return torch.nn.functional.gelu(x, approximate="tanh")
    if act == 2:
        return torch.relu(x)
    if act == 3:
        return torch.nn.functional.silu(x)
    return x


class Deadlock(RuntimeError):
    pass


class RaceDetected(RuntimeError):
    pass


class RedundantOp(ValueError):
    """A plan op that repeats the previous op of its stream exactly (same flags, same value):
    a wasted launch / memop per run that the executor would faithfully enqueue."""


def check_redundant(plan: Plan) -> None:
    """Flag identical back-to-back signals on one stream (e.g. a copy-paste duplicate of an
    arrival signal): raises :class:`RedundantOp`."""
    last: Dict[int, object] = {}
    for i, op in enumerate(plan.ops):
        prev = last.get(op.stream)
        if (op.kind == OP_SIGNAL and prev is not None and prev.kind == OP_SIGNAL
                and prev.args == op.args):
            raise RedundantOp(f"op {i} (stream {op.stream}) repeats the signal before it: "
                              f"{[f'{f.buf}+{f.off}' for f in op.args['flags']]}")
        last[op.stream] = op


def _view(buf: torch.Tensor, off: int, count: int, dt: int) -> torch.Tensor:
    es = DT_SIZE[dt]
    return buf[off:off + count * es].view(TORCH_DT[dt])


class _VC:
    __slots__ = ("v",)

    def __init__(self, n: int):
        self.v = [0] * n

    def join(self, other: "_VC") -> None:
        self.v = [max(a, b) for a, b in zip(self.v, other.v)]

    def copy(self) -> "_VC":
        c = _VC(0)
        c.v = list(self.v)
        return c

    def leq(self, other: "_VC") -> bool:
        return all(a <= b for a, b in zip(self.v, other.v))


class Simulator:
    def __init__(self, plans: Sequence[Plan], buffers: Sequence[Dict[str, torch.Tensor]],
                 check_races: bool = True):
        self.plans = list(plans)
        for p in self.plans:
            check_redundant(p)
        self.d = len(plans)
        self.bufs = list(buffers)
        self.check_races = check_races
        self.nstreams = max(p.nstreams for p in plans)
        self.epoch = [0] * self.d
        self.flag_bufs = {name for p in plans for name, b in p.buffers.items()
                          if b.symmetric and b.zero}
        self.accesses: Dict[Tuple[int, str], List] = {}
        self._comp = lambda r, s: r * self.nstreams + s
        self.rank_vc = [_VC(self.d * self.nstreams) for _ in range(self.d)]
        self.flag_vc: Dict = {}

    # --------------------------------------------------------------- memory helpers
    def _owner(self, rank: int, ref: Ref) -> int:
        return rank if ref.owner is None else ref.owner

    def _buf(self, rank: int, ref: Ref) -> torch.Tensor:
        return self.bufs[self._owner(rank, ref)][ref.buf]

    def _touch(self, rank, ref: Ref, nbytes: int, write: bool, vc: _VC, what: str):
        if not self.check_races or ref.buf in self.flag_bufs or nbytes <= 0:
            return
        owner = self._owner(rank, ref)
        key = (owner, ref.buf)
        lo, hi = ref.off, ref.off + nbytes
        log = self.accesses.setdefault(key, [])
        for (plo, phi, pw, pvc, pwhat) in log:
            if plo < hi and lo < phi and (pw or write) and not pvc.leq(vc):
                raise RaceDetected(
                    f"race on rank {owner} buffer {ref.buf} bytes [{max(lo, plo)},{min(hi, phi)}): "
                    f"{pwhat} vs {what} (not ordered by happens-before)")
        log.append((lo, hi, write, vc.copy(), what))
        if len(log) > 4000:
            del log[:2000]

    # --------------------------------------------------------------- op semantics
    def _rows(self, base: Ref, M: int, grp: int, gstride: int, ld: int, width: int, es: int):
        """Byte ranges (Ref, nbytes) of the rows a grouped mapping touches."""
        if grp <= 0:
            grp, gstride = max(M, 1), max(M, 1)
        out = []
        g = 0
        while g * grp < M:
            rows = min(grp, M - g * grp)
            start = base + (g * gstride) * ld * es
            out.append((start, ((rows - 1) * ld + width) * es))
            g += 1
        return out

    def _gather_rows(self, buf, off, M, grp, gstride, ld, width, dt):
        es = DT_SIZE[dt]
        if grp <= 0:
            grp, gstride = max(M, 1), max(M, 1)
        idx = torch.arange(M)
        phys = (idx // grp) * gstride + (idx % grp)
        need = int(phys.max().item()) * ld + width if M else 0
        flat = _view(buf, off, need, dt)
        rows = flat.as_strided((int(phys.max().item()) + 1, width), (ld, 1))
        return rows[phys]

    def _scatter_rows(self, buf, off, M, grp, gstride, ld, width, dt, values):
        if grp <= 0:
            grp, gstride = max(M, 1), max(M, 1)
        idx = torch.arange(M)
        phys = (idx // grp) * gstride + (idx % grp)
        need = int(phys.max().item()) * ld + width
        flat = _view(buf, off, need, dt)
        rows = flat.as_strided((int(phys.max().item()) + 1, width), (ld, 1))
        rows[phys] = values.to(TORCH_DT[dt])

    def _exec_local(self, r: int, op, vc: _VC) -> None:
        a, k = op.args, op.kind
        what = f"r{r}.s{op.stream}.{OP_NAMES[k]}"
        if k == OP_GEMM and a.get("ag") is not None:
            self._exec_ag(r, op, vc, what)
        if k == OP_GEMM and a.get("ksplit", 1) > 1:
            # K-split: slice s = A / B columns [s K, (s + 1) K) -> partial s at c + s * M * ldc
            ein, eout = DT_SIZE[a["din"]], DT_SIZE[a["dout"]]
            for sl in range(a["ksplit"]):
                sub = dict(a, ksplit=1, a=a["a"] + sl * a["K"] * ein, b=a["b"] + sl * a["K"] * ein,
                           c=a["c"] + sl * a["M"] * a["ldc"] * eout)
                self._exec_local(r, type(op)(k, op.stream, sub), vc)
            return
        if k == OP_GEMM:
            ein, eout = DT_SIZE[a["din"]], DT_SIZE[a["dout"]]
            shards = a.get("a_shards")
            if shards is not None:  # direct-access GEMM: row block s read from a_shards[s]
                R, parts = a["shard_rows"], []
                for sidx, ref in enumerate(shards):
                    rows = min(R, a["M"] - sidx * R)
                    if rows <= 0:
                        break
                    span = (rows - 1) * a["lda"] + a["K"]
                    self._touch(r, ref, span * ein, False, vc, what + f".A{sidx}")
                    parts.append(_view(self._buf(r, ref), ref.off, span, a["din"]).as_strided(
                        (rows, a["K"]), (a["lda"], 1)).float())
                A_shards = torch.cat(parts)
            else:
                A_shards = None
                for ref, nb in self._rows(a["a"], a["M"], a["a_grp"], a["a_gstride"], a["lda"],
                                          a["K"], ein):
                    self._touch(r, ref, nb, False, vc, what + ".A")
            self._touch(r, a["b"], ((a["N"] - 1) * a["ldb"] + a["K"]) * ein, False, vc, what + ".B")
            cshards = a.get("c_shards")
            if cshards is None:
                for ref, nb in self._rows(a["c"], a["M"], a["c_grp"], a["c_gstride"], a["ldc"],
                                          a["N"], eout):
                    self._touch(r, ref, nb, True, vc, what + ".C")
            A = A_shards if A_shards is not None else self._gather_rows(
                self._buf(r, a["a"]), a["a"].off, a["M"], a["a_grp"], a["a_gstride"], a["lda"],
                a["K"], a["din"]).float()
            Bt = _view(self._buf(r, a["b"]), a["b"].off, (a["N"] - 1) * a["ldb"] + a["K"],
                       a["din"]).as_strided((a["N"], a["K"]), (a["ldb"], 1)).float()
            Cv = apply_act(A @ Bt.t(), a.get("act", 0))
            if cshards is None:
                self._scatter_rows(self._buf(r, a["c"]), a["c"].off, a["M"], a["c_grp"],
                                   a["c_gstride"], a["ldc"], a["N"], a["dout"], Cv)
            else:  # direct-store C: row block s written at c_shards[s] (maybe a peer's buffer)
                R = a["c_shard_rows"]
                for sidx, ref in enumerate(cshards):
                    rows = min(R, a["M"] - sidx * R)
                    if rows <= 0:
                        break
                    self._touch(r, ref, ((rows - 1) * a["ldc"] + a["N"]) * eout, True, vc,
                                what + f".C{sidx}")
                    self._scatter_rows(self._buf(r, ref), ref.off, rows, 0, 0, a["ldc"], a["N"],
                                       a["dout"], Cv[sidx * R:sidx * R + rows])
        elif k == OP_COPY:
            self._touch(r, a["src"], a["nbytes"], False, vc, what + ".src")
            self._touch(r, a["dst"], a["nbytes"], True, vc, what + ".dst")
            src = self._buf(r, a["src"])[a["src"].off:a["src"].off + a["nbytes"]]
            self._buf(r, a["dst"])[a["dst"].off:a["dst"].off + a["nbytes"]] = src
        elif k in (OP_COPY_MULTI, OP_COPY_BATCH):
            for (dst, src, nb) in a["segs"]:
                self._touch(r, src, nb, False, vc, what + ".src")
                self._touch(r, dst, nb, True, vc, what + ".dst")
                self._buf(r, dst)[dst.off:dst.off + nb] = self._buf(r, src)[src.off:src.off + nb]
        elif k == OP_REDUCE:
            es = DT_SIZE[a["dtype"]]
            acc = None
            for s in a["srcs"]:
                self._touch(r, s, a["count"] * es, False, vc, what + ".src")
                x = _view(self._buf(r, s), s.off, a["count"], a["dtype"]).float()
                acc = x.clone() if acc is None else acc + x
            self._touch(r, a["dst"], a["count"] * es, True, vc, what + ".dst")
            _view(self._buf(r, a["dst"]), a["dst"].off, a["count"], a["dtype"])[:] = acc.to(
                TORCH_DT[a["dtype"]])
        elif k == OP_MEMSET:
            self._touch(r, a["dst"], a["nbytes"], True, vc, what)
            self._buf(r, a["dst"])[a["dst"].off:a["dst"].off + a["nbytes"]] = a["value"]
        elif k == OP_SIGNAL:
            val = self.epoch[r] + a["delta"]
            for f in a["flags"]:
                buf = self._buf(r, f)
                buf[f.off:f.off + 4].view(torch.int32)[0] = val
                self.flag_vc[(self._owner(r, f), f.buf, f.off, val)] = vc.copy()
        elif k in (OP_RECORD, OP_WAIT, OP_WAIT_SIGNAL, OP_NOP):
            pass
        else:
            raise AssertionError(f"not a local op: {OP_NAMES[k]}")

    def _exec_ag(self, r: int, op, vc: _VC, what: str) -> None:
        """Copy workgroups of an in-kernel all-gather: every peer's row blocks into the same
        rows of A, each block's ARRIVE flag, then an ACK at the producer."""
        a = op.args
        g = a["ag"]
        npro, nsub = a["nshards"] // a["nsub"], a["nsub"]
        seg = a["flag_rows"] * a["lda"] * DT_SIZE[a["din"]]
        val = self.epoch[r]
        for q in range(npro):
            if q == g["rank"]:
                continue
            for b in range(nsub):
                off = (q * nsub + b) * seg
                src, dst = g["src"][q] + off, a["a"] + off
                self._touch(r, src, seg, False, vc, what + f".ag.src{q}")
                self._touch(r, dst, seg, True, vc, what + ".ag.dst")
                self._buf(r, dst)[dst.off:dst.off + seg] = \
                    self._buf(r, src)[src.off:src.off + seg].clone()
                f = a["flags"] + 4 * (q * nsub + b)
                self._buf(r, f)[f.off:f.off + 4].view(torch.int32)[0] = val
                self.flag_vc[(self._owner(r, f), f.buf, f.off, val)] = vc.copy()
            f = g["ack"][q]
            self._buf(r, f)[f.off:f.off + 4].view(torch.int32)[0] = val
            self.flag_vc[(self._owner(r, f), f.buf, f.off, val)] = vc.copy()

    # --------------------------------------------------------------- collectives
    def _exec_collective(self, group: List[Tuple[int, List]], vcs: List[_VC]) -> None:
        """group = [(rank, [ops]) ...] for every rank; ops = one collective or a send/recv group."""
        kinds = {tuple(o.kind for o in ops) for _, ops in group}
        first = group[0][1][0]
        if first.kind == OP_ALLGATHER:
            a0 = first.args
            es = DT_SIZE[a0["dtype"]]
            nb = a0["count"] * es
            snaps = []
            for (r, ops), vc in zip(group, vcs):
                a = ops[0].args
                self._touch(r, a["send"], nb, False, vc, f"r{r}.allgather.send")
                snaps.append(self._buf(r, a["send"])[a["send"].off:a["send"].off + nb].clone())
            for (r, ops), vc in zip(group, vcs):
                a = ops[0].args
                self._touch(r, a["recv"], nb * self.d, True, vc, f"r{r}.allgather.recv")
                buf = self._buf(r, a["recv"])
                for q in range(self.d):
                    buf[a["recv"].off + q * nb:a["recv"].off + (q + 1) * nb] = snaps[q]
        elif first.kind == OP_REDUCE_SCATTER:
            a0 = first.args
            dt = a0["dtype"]
            cnt = a0["count"]
            ins = []
            for (r, ops), vc in zip(group, vcs):
                a = ops[0].args
                self._touch(r, a["send"], cnt * self.d * DT_SIZE[dt], False, vc, f"r{r}.rs.send")
                ins.append(_view(self._buf(r, a["send"]), a["send"].off, cnt * self.d, dt).float())
            total = torch.stack(ins).sum(0)
            for (r, ops), vc in zip(group, vcs):
                a = ops[0].args
                self._touch(r, a["recv"], cnt * DT_SIZE[dt], True, vc, f"r{r}.rs.recv")
                _view(self._buf(r, a["recv"]), a["recv"].off, cnt, dt)[:] = \
                    total[r * cnt:(r + 1) * cnt].to(TORCH_DT[dt])
        else:  # send/recv group
            sends: Dict[Tuple[int, int], List] = {}
            for (r, ops), vc in zip(group, vcs):
                for o in ops:
                    if o.kind == OP_SEND:
                        a = o.args
                        nb = a["count"] * DT_SIZE[a["dtype"]]
                        self._touch(r, a["buf"], nb, False, vc, f"r{r}.send")
                        data = self._buf(r, a["buf"])[a["buf"].off:a["buf"].off + nb].clone()
                        sends.setdefault((r, a["peer"]), []).append(data)
            for (r, ops), vc in zip(group, vcs):
                for o in ops:
                    if o.kind == OP_RECV:
                        a = o.args
                        nb = a["count"] * DT_SIZE[a["dtype"]]
                        q = sends.get((a["peer"], r))
                        if not q:
                            raise Deadlock(f"rank {r} recv from {a['peer']} has no matching send")
                        data = q.pop(0)
                        if data.numel() != nb:
                            raise RuntimeError("send/recv size mismatch")
                        self._touch(r, a["buf"], nb, True, vc, f"r{r}.recv")
                        self._buf(r, a["buf"])[a["buf"].off:a["buf"].off + nb] = data
            left = {k: v for k, v in sends.items() if v}
            if left:
                raise Deadlock(f"unmatched sends {list(left)}")
        del kinds

    # --------------------------------------------------------------- scheduler
    def run_epoch(self) -> None:
        """Run one epoch on every rank (all ranks advance one epoch)."""
        d = self.d
        for r in range(d):
            self.epoch[r] += 1
        # split each rank's ops into per-stream queues; group send/recv and collectives
        queues: List[List[List]] = []
        coll_seq: List[List] = []
        for r, plan in enumerate(self.plans):
            qs: List[List] = [[] for _ in range(plan.nstreams)]
            seq = 0
            i = 0
            ops = plan.ops
            while i < len(ops):
                op = ops[i]
                if op.kind == OP_GROUP_START:
                    j = i + 1
                    grp = []
                    while ops[j].kind != OP_GROUP_END:
                        grp.append(ops[j])
                        j += 1
                    qs[op.stream].append(("coll", seq, grp, op.stream))
                    seq += 1
                    i = j + 1
                    continue
                if op.kind in (OP_ALLGATHER, OP_REDUCE_SCATTER):
                    qs[op.stream].append(("coll", seq, [op], op.stream))
                    seq += 1
                elif op.kind in (OP_SEND, OP_RECV):
                    qs[op.stream].append(("coll", seq, [op], op.stream))
                    seq += 1
                else:
                    qs[op.stream].append(("op", i, op, op.stream))
                i += 1
            queues.append(qs)
        heads = [[0] * len(q) for q in queues]
        # per rank: last record op index per event (issue order) -> executed flag
        recorded: List[Dict[int, _VC]] = [dict() for _ in range(d)]
        record_issue: List[Dict[int, int]] = [dict() for _ in range(d)]
        wait_target: List[Dict[int, Optional[int]]] = [dict() for _ in range(d)]
        for r, plan in enumerate(self.plans):
            last: Dict[int, int] = {}
            for i, op in enumerate(plan.ops):
                if op.kind == OP_RECORD:
                    last[op.args["event"]] = i
                elif op.kind == OP_WAIT:
                    wait_target[r][i] = last.get(op.args["event"])
        done_rec: List[Dict[int, _VC]] = [dict() for _ in range(d)]
        stream_vc = [[self.rank_vc[r].copy() for _ in range(self.nstreams)] for r in range(d)]
        pending = sum(len(q) for qs in queues for q in qs)
        while pending:
            progressed = False
            # collectives: ready when every rank has the same seq at the head of a stream
            heads_coll = {}
            for r in range(d):
                for s, q in enumerate(queues[r]):
                    h = heads[r][s]
                    if h < len(q) and q[h][0] == "coll":
                        heads_coll[r] = (q[h][1], s, q[h][2])
            if len(heads_coll) == d and len({v[0] for v in heads_coll.values()}) == 1:
                vcs = []
                for r in range(d):
                    seq, s, grp = heads_coll[r]
                    vcs.append(stream_vc[r][s].copy())
                joined = vcs[0].copy()
                for v in vcs[1:]:
                    joined.join(v)
                self._exec_collective([(r, heads_coll[r][2]) for r in range(d)],
                                      [joined] * d)
                for r in range(d):
                    s = heads_coll[r][1]
                    nv = joined.copy()
                    nv.v[self._comp(r, s)] += 1
                    stream_vc[r][s] = nv
                    heads[r][s] += 1
                    pending -= 1
                progressed = True
                continue
            for r in range(d):
                for s, q in enumerate(queues[r]):
                    while heads[r][s] < len(q) and q[heads[r][s]][0] == "op":
                        _, idx, op, _ = q[heads[r][s]]
                        vc = stream_vc[r][s].copy()
                        if op.kind == OP_WAIT:
                            tgt = wait_target[r].get(idx)
                            if tgt is not None:
                                if tgt not in done_rec[r]:
                                    break
                                vc.join(done_rec[r][tgt])
                        elif op.kind == OP_GEMM and op.args.get("ag") is not None:
                            # in-kernel all-gather: the copy workgroups read producer p only
                            # after READY[p]; the own blocks' flags come from earlier ops. The
                            # launch is modelled atomically: copies, flags, ACKs, then the GEMM
                            a = op.args
                            g = a["ag"]
                            npro = a["nshards"] // a["nsub"]
                            gate = [g["ready"] + 4 * q for q in range(npro) if q != g["rank"]]
                            gate += [a["flags"] + 4 * (g["rank"] * a["nsub"] + b)
                                     for b in range(a["nsub"])]
                            ok = True
                            for f in gate:
                                val = int(self._buf(r, f)[f.off:f.off + 4].view(torch.int32)[0])
                                if val < self.epoch[r]:
                                    ok = False
                                    break
                                src = self.flag_vc.get((self._owner(r, f), f.buf, f.off, val))
                                if src is not None:
                                    vc.join(src)
                            if not ok:
                                break
                        elif op.kind == OP_GEMM and op.args.get("flags") is not None:
                            # flag-gated GEMM: every tile spins on flags[shard] >= epoch before
                            # reading its A rows; atomically modelled as waiting on all shards
                            a = op.args
                            base = a["flags"]
                            ok = True
                            for sh in range(a["nshards"]):
                                if (a.get("tile_order") == 3
                                        and sh // a["nsub"] == a["first_shard"]):
                                    continue  # own rows: never gated (csrc wait_flag_t0)
                                f = base + 4 * sh
                                val = int(self._buf(r, f)[f.off:f.off + 4].view(torch.int32)[0])
                                if val < self.epoch[r]:
                                    ok = False
                                    break
                                src = self.flag_vc.get((self._owner(r, f), f.buf, f.off, val))
                                if src is not None:
                                    vc.join(src)
                            if not ok:
                                break
                        elif op.kind == OP_WAIT_SIGNAL:
                            need = self.epoch[r] + op.args["delta"]
                            ok = True
                            for f in op.args["flags"]:
                                buf = self._buf(r, f)
                                val = int(buf[f.off:f.off + 4].view(torch.int32)[0])
                                if need > 0 and val < need:
                                    ok = False
                                    break
                                if need > 0:
                                    src = self.flag_vc.get((self._owner(r, f), f.buf, f.off, val))
                                    if src is not None:
                                        vc.join(src)
                            if not ok:
                                break
                        vc.v[self._comp(r, s)] += 1
                        self._exec_local(r, op, vc)
                        if op.kind == OP_RECORD:
                            done_rec[r][idx] = vc.copy()
                        stream_vc[r][s] = vc
                        heads[r][s] += 1
                        pending -= 1
                        progressed = True
            if not progressed:
                stuck = []
                for r in range(d):
                    for s, q in enumerate(queues[r]):
                        h = heads[r][s]
                        if h < len(q):
                            item = q[h]
                            desc = (OP_NAMES[item[2].kind] if item[0] == "op"
                                    else "coll#" + str(item[1]))
                            stuck.append(f"rank {r} stream {s}: {desc}")
                raise Deadlock("plan deadlocks at epoch %d:\n  " % self.epoch[0] +
                               "\n  ".join(stuck))
        # join: every stream of a rank precedes the next epoch
        for r in range(d):
            v = self.rank_vc[r].copy()
            for s in range(self.nstreams):
                v.join(stream_vc[r][s])
            self.rank_vc[r] = v


def make_buffers(plans: Sequence[Plan]) -> List[Dict[str, torch.Tensor]]:
    out = []
    for p in plans:
        bufs = {}
        for name, spec in p.buffers.items():
            bufs[name] = torch.zeros(spec.nbytes, dtype=torch.uint8)
        out.append(bufs)
    return out


def write_tensor(bufs: Dict[str, torch.Tensor], loc, tensor: torch.Tensor) -> None:
    es = DT_SIZE[loc.dtype]
    flat = tensor.contiguous().view(-1).view(torch.uint8) if tensor.dtype != torch.uint8 else \
        tensor.contiguous().view(-1)
    n = loc.rows * loc.cols * es
    bufs[loc.buf][loc.off:loc.off + n] = flat[:n]


def read_tensor(bufs: Dict[str, torch.Tensor], loc) -> torch.Tensor:
    es = DT_SIZE[loc.dtype]
    n = loc.rows * loc.cols * es
    return bufs[loc.buf][loc.off:loc.off + n].view(TORCH_DT[loc.dtype]).view(loc.rows, loc.cols)
