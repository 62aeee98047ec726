"""Every native algorithm, simulated on the CPU for d ranks: layout math, synchronisation
protocol (no deadlock, no unordered conflicting access) and numerics vs an fp32 reference."""

import itertools
import math

import pytest
import torch

from ddlb_amd.parallel.algorithms import S_COMM, AlgoConfig, build_tp_columnwise, build_tp_rowwise
from ddlb_amd.parallel.plan import (DT_BF16, DT_F32, OP_COPY, OP_COPY_MULTI, OP_GEMM, OP_RECORD,
                                    OP_REDUCE, OP_SIGNAL, OP_WAIT, SIG_KERNEL, SIG_STREAM)
from ddlb_amd.parallel.sim import Simulator, make_buffers, read_tensor, write_tensor

ALGS = ["default", "coll_pipeline", "p2p_pipeline"]
BACKENDS = ["rccl", "ipc"]
PROTOCOLS = ["memcpy", "batch_memcpy", "kernel"]


def _inputs(m, n, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    A = torch.randint(-3, 4, (m, k), generator=g).float()
    B = torch.randint(-3, 4, (k, n), generator=g).float()
    return A, B


def _run_col(d, m, n, k, cfg, epochs=3, dt=DT_F32):
    A, B = _inputs(m, n, k)
    tdt = torch.float32 if dt == DT_F32 else torch.bfloat16
    built = [build_tp_columnwise(r, d, m, n, k, dt, dt, cfg) for r in range(d)]
    plans = [p for p, _ in built]
    bufs = make_buffers(plans)
    ml = m // d
    for r, (_, io) in enumerate(built):
        write_tensor(bufs[r], io.a, A[r * ml:(r + 1) * ml].to(tdt))
        write_tensor(bufs[r], io.b, B.t().contiguous().to(tdt))
    sim = Simulator(plans, bufs)
    for _ in range(epochs):
        sim.run_epoch()
    ref = A @ B
    for r, (_, io) in enumerate(built):
        out = read_tensor(bufs[r], io.out).float()
        torch.testing.assert_close(out, ref, rtol=0, atol=0)


def _run_row(d, m, n, k, cfg, epochs=3, dt=DT_F32):
    A, B = _inputs(m, n, k, seed=1)
    tdt = torch.float32 if dt == DT_F32 else torch.bfloat16
    built = [build_tp_rowwise(r, d, m, n, k, dt, dt, cfg) for r in range(d)]
    plans = [p for p, _ in built]
    bufs = make_buffers(plans)
    kl, ml = k // d, m // d
    for r, (_, io) in enumerate(built):
        write_tensor(bufs[r], io.a, A[:, r * kl:(r + 1) * kl].contiguous().to(tdt))
        write_tensor(bufs[r], io.b, B[r * kl:(r + 1) * kl].t().contiguous().to(tdt))
    sim = Simulator(plans, bufs)
    for _ in range(epochs):
        sim.run_epoch()
    ref = A @ B
    for r, (_, io) in enumerate(built):
        out = read_tensor(bufs[r], io.out).float()
        torch.testing.assert_close(out, ref[r * ml:(r + 1) * ml], rtol=0, atol=0)


@pytest.mark.parametrize("d", [1, 2, 3, 4])
@pytest.mark.parametrize("alg,backend", list(itertools.product(ALGS, BACKENDS)))
@pytest.mark.parametrize("order", ["AG_before", "AG_after"])
def test_columnwise_plans(d, alg, backend, order):
    cfg = AlgoConfig(algorithm=alg, backend=backend, order=order, s=2)
    _run_col(d, m=16 * d, n=8, k=12, cfg=cfg)


@pytest.mark.parametrize("d", [1, 2, 3, 4])
@pytest.mark.parametrize("alg,backend", list(itertools.product(ALGS, BACKENDS)))
def test_rowwise_plans(d, alg, backend):
    cfg = AlgoConfig(algorithm=alg, backend=backend, s=2)
    _run_row(d, m=16 * d, n=8, k=4 * d, cfg=cfg)


@pytest.mark.parametrize("protocol", PROTOCOLS)
@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("ring", [True, False])
@pytest.mark.parametrize("sig", [SIG_STREAM, SIG_KERNEL])
def test_ipc_protocols(protocol, alg, ring, sig):
    cfg = AlgoConfig(algorithm=alg, backend="ipc", protocol=protocol, ring=ring, signal=sig, s=2,
                     inter_stream_sync=ring)
    _run_col(3, m=24, n=8, k=8, cfg=cfg)
    _run_row(3, m=24, n=8, k=9, cfg=cfg)


@pytest.mark.parametrize("d", [2, 3, 4])
@pytest.mark.parametrize("protocol", PROTOCOLS)
@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("sig", [SIG_STREAM, SIG_KERNEL])
def test_ipc_push_plans(d, protocol, alg, sig):
    """direction=push: writers fill every peer's gather buffer; arrival flags / ACK epochs."""
    cfg = AlgoConfig(algorithm=alg, backend="ipc", protocol=protocol, signal=sig, s=2,
                     direction="push")
    _run_col(d, 8 * d, 8, 8, cfg, epochs=4)


def test_push_rejected_where_meaningless():
    for cfg in (AlgoConfig(algorithm="default", backend="rccl", direction="push"),
                AlgoConfig(algorithm="direct", backend="ipc", direction="push"),
                AlgoConfig(algorithm="p2p_pipeline", backend="ipc", fused=True, direction="push"),
                AlgoConfig(backend="ipc", order="AG_after", direction="push")):
        with pytest.raises(ValueError):
            build_tp_columnwise(0, 2, 16, 8, 8, DT_F32, DT_F32, cfg)
    with pytest.raises(ValueError):
        build_tp_rowwise(0, 2, 16, 8, 8, DT_F32, DT_F32, AlgoConfig(backend="ipc",
                                                                     direction="push"))


@pytest.mark.parametrize("alg,backend", [("coll_pipeline", "ipc"), ("default", "ipc"),
                                         ("p2p_pipeline", "rccl")])
def test_rowwise_rejects_fused(alg, backend):
    """tp_rowwise fused = the direct-store p2p_pipeline over IPC only; anything else must be
    refused up front, not fail while building."""
    cfg = AlgoConfig(algorithm=alg, backend=backend, s=2, fused=True)
    with pytest.raises(ValueError, match="direct-store"):
        build_tp_rowwise(0, 2, 16, 8, 8, DT_F32, DT_F32, cfg)


@pytest.mark.parametrize("d", [1, 2, 3, 4])
@pytest.mark.parametrize("sig", [SIG_STREAM, SIG_KERNEL])
def test_rowwise_direct_store_plan(d, sig):
    """tp_rowwise p2p_pipeline fused: ONE GEMM whose row block q lands in rank q's receive slot
    (direct store over xGMI), interleaved shard order; READY / reduce / ACK epochs."""
    cfg = AlgoConfig(algorithm="p2p_pipeline", backend="ipc", fused=True, signal=sig)
    _run_row(d, m=8 * d, n=8, k=4 * d, cfg=cfg, epochs=4)
    if d > 1:
        plan, _ = build_tp_rowwise(1, d, 8 * d, 8, 4 * d, DT_F32, DT_F32, cfg)
        g = [op for op in plan.ops if op.kind == OP_GEMM]
        assert len(g) == 1 and g[0].args["tile_order"] == 2 and g[0].args["c_shard_rows"] == 8
        owners = [ref.owner for ref in g[0].args["c_shards"]]
        assert owners == [q if q != 1 else None for q in range(d)]


@pytest.mark.parametrize("fused", [True, False])
def test_p2p_fused_plan(fused):
    cfg = AlgoConfig(algorithm="p2p_pipeline", backend="ipc", fused=fused)
    _run_col(4, m=32, n=8, k=8, cfg=cfg)


@pytest.mark.parametrize("d", [2, 3, 4])
@pytest.mark.parametrize("sig", [SIG_STREAM, SIG_KERNEL])
@pytest.mark.parametrize("protocol", ["memcpy", "batch_memcpy"])
def test_coll_fused_plan(d, sig, protocol):
    """coll_pipeline fused: one flag-gated GEMM, ARRIVE per (peer, block), block-major order."""
    cfg = AlgoConfig(algorithm="coll_pipeline", backend="ipc", fused=True, s=3, signal=sig,
                     protocol=protocol)
    _run_col(d, m=6 * d, n=8, k=8, cfg=cfg, epochs=3)
    plan, _ = build_tp_columnwise(1, d, 6 * d, 8, 8, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == 1 and g[0].args["nshards"] == 3 * d and g[0].args["nsub"] == 3
    assert g[0].args["flag_rows"] == 2 and g[0].args["first_shard"] == 1


def test_fused_rejected_where_meaningless():
    for cfg in (AlgoConfig(algorithm="default", backend="ipc", fused=True),
                AlgoConfig(algorithm="default", backend="rccl", fused=True),
                AlgoConfig(algorithm="coll_pipeline", backend="rccl", order="AG_after",
                           fused=True),
                AlgoConfig(algorithm="p2p_pipeline", backend="ipc", order="AG_after",
                           fused=True)):
        with pytest.raises(ValueError):
            build_tp_columnwise(0, 2, 16, 8, 8, DT_F32, DT_F32, cfg)


@pytest.mark.parametrize("d", [2, 3, 4, 8])
@pytest.mark.parametrize("s", [1, 2, 8])
def test_rccl_fused_coll_plan(d, s):
    """coll_pipeline over RCCL feeding ONE gated GEMM: stage-major gather buffer, A through a
    row-block table (own blocks read in place), local ARRIVE flags raised by signal kernels after
    each stage's all-gather, own blocks dispatched first (tile_order 3)."""
    cfg = AlgoConfig(algorithm="coll_pipeline", backend="rccl", fused=True, s=s)
    _run_col(d, m=2 * d * s, n=8, k=12, cfg=cfg, epochs=3)
    rank = 1
    plan, io = build_tp_columnwise(rank, d, 2 * d * s, 8, 12, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == 1 and g[0].args["M"] == 2 * d * s and g[0].args["tile_order"] == 3
    assert g[0].args["nshards"] == d * s and g[0].args["nsub"] == s
    assert g[0].args["first_shard"] == rank and g[0].args["shard_rows"] == 2
    tab = g[0].args["a_shards"]
    assert [t.buf for t in tab[rank * s:(rank + 1) * s]] == ["A_full"] * s
    assert all(t.buf == "G" for i, t in enumerate(tab) if i // s != rank)
    assert not plan.buffers["flags"].symmetric
    sigs = [op for op in plan.ops if op.kind == OP_SIGNAL and op.stream == S_COMM]
    assert all(op.args["method"] == SIG_KERNEL for op in sigs) and len(sigs) >= s


@pytest.mark.parametrize("d", [2, 3, 4, 8])
def test_rccl_fused_p2p_plan(d):
    """p2p_pipeline over RCCL send / recv feeding ONE gated GEMM (shard order from the own)."""
    cfg = AlgoConfig(algorithm="p2p_pipeline", backend="rccl", fused=True)
    _run_col(d, m=4 * d, n=8, k=12, cfg=cfg, epochs=3)
    plan, _ = build_tp_columnwise(0, d, 4 * d, 8, 12, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == 1 and g[0].args["nshards"] == d and g[0].args["flags"] is not None


def test_rccl_fused_coll_negative_no_signal():
    """Without the stage signal kernels the gated GEMM can never see the peers' blocks."""
    from ddlb_amd.parallel.sim import Deadlock

    cfg = AlgoConfig(algorithm="coll_pipeline", backend="rccl", fused=True, s=2)
    built = [build_tp_columnwise(r, 2, 8, 8, 8, DT_F32, DT_F32, cfg) for r in range(2)]
    plans = [p for p, _ in built]
    for p in plans:
        p.ops = [op for op in p.ops if op.kind != OP_SIGNAL]
    sim = Simulator(plans, make_buffers(plans))
    with pytest.raises(Deadlock):
        sim.run_epoch()


@pytest.mark.parametrize("d", [1, 2, 3, 4])
@pytest.mark.parametrize("sig", [SIG_STREAM, SIG_KERNEL])
def test_direct_access_plans(d, sig):
    """algorithm=direct: one GEMM reading every peer's shard in place (no gather buffer)."""
    cfg = AlgoConfig(algorithm="direct", backend="ipc", signal=sig)
    _run_col(d, m=12 * d, n=8, k=8, cfg=cfg)


def test_direct_access_rejects_bad_configs():
    with pytest.raises(ValueError):
        build_tp_columnwise(0, 2, 16, 8, 8, DT_F32, DT_F32, AlgoConfig(algorithm="direct"))
    with pytest.raises(ValueError):
        build_tp_rowwise(0, 2, 16, 8, 8, DT_F32, DT_F32,
                         AlgoConfig(algorithm="direct", backend="ipc"))


def test_bf16_plans_round_like_hardware():
    cfg = AlgoConfig(algorithm="coll_pipeline", backend="rccl", s=2)
    _run_col(2, m=16, n=8, k=8, cfg=cfg, dt=DT_BF16)


def test_invalid_configs():
    with pytest.raises(ValueError):
        build_tp_columnwise(0, 2, 30, 8, 8, DT_F32, DT_F32, AlgoConfig(algorithm="coll_pipeline", s=4))
    with pytest.raises(ValueError):
        build_tp_rowwise(0, 2, 16, 8, 7, DT_F32, DT_F32, AlgoConfig())


def _bench_native_cfgs():
    """(primitive, label, AlgoConfig) of every native candidate bench.py can pick at world > 1
    (the default pool and the --candidates extras)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from ddlb_amd.primitives.native_common import algo_config
    from ddlb_amd.primitives.registry import resolve

    out = []
    for prim in ("tp_columnwise", "tp_rowwise"):
        for label, impl, opts in bench.candidate_pool(prim, "bfloat16", 8, extra=True):
            if impl != "native":
                continue
            cls, o, _ = resolve(prim, impl, dict(opts))
            merged = {**cls.DEFAULT_OPTIONS, **o}
            for key, alias in cls.OPTION_ALIASES.items():
                merged[key] = alias.get(merged[key], merged[key])
            out.append((prim, label, algo_config(merged, order=merged.get("order", "AG_before"))))
    return out


@pytest.mark.parametrize("d", [2, 4, 8])
@pytest.mark.parametrize("prim,label,cfg", _bench_native_cfgs(),
                         ids=[c[1] for c in _bench_native_cfgs()])
def test_bench_candidates_simulate(d, prim, label, cfg):
    """Every native candidate of the N>1 bench pool, at the driver's world sizes (incl. 8, which
    no GPU box here can run): protocol completes, no race, exact result, several epochs."""
    s = cfg.s if cfg.algorithm == "coll_pipeline" else 1
    if prim == "tp_columnwise" and cfg.fused and cfg.protocol == "kernel":
        # in-kernel all-gather: the persistent 256x256 kernel's shape rules
        _run_col(d, m=256 * d * s // math.gcd(256, d * s), n=256, k=64, cfg=cfg, epochs=2)
    elif prim == "tp_columnwise":
        _run_col(d, m=4 * d * s, n=8, k=12, cfg=cfg, epochs=2)
    else:
        _run_row(d, m=4 * d * s, n=8, k=4 * d, cfg=cfg, epochs=2)


def test_format_timeline_text():
    from ddlb_amd.parallel.explain import format_timeline

    rows = [{"index": 0, "op": "wait_signal", "stream": 2, "start_ms": 0.0, "end_ms": 0.01},
            {"index": 1, "op": "copy", "stream": 2, "start_ms": 0.01, "end_ms": 0.05},
            {"index": 2, "op": "gemm", "stream": 0, "start_ms": 0.0, "end_ms": 0.04},
            {"index": 3, "op": "wait", "stream": 0, "start_ms": 0.04, "end_ms": 0.05},
            {"index": 4, "op": "gemm", "stream": 0, "start_ms": 0.05, "end_ms": 0.08}]
    text = format_timeline(rows, width=40)
    assert "80.0 us" in text and "s0" in text and "s2" in text
    bars = [ln for ln in text.splitlines() if ln.lstrip().startswith("s")]
    assert "G" in bars[0] and "c" in bars[1] and "w" in bars[1]
    ratio = float(text.split("busy time over streams / span = ")[1].split()[0])
    assert abs(ratio - (40 + 30 + 40) / 80) < 0.01


@pytest.mark.parametrize("d", [2, 3, 4])
@pytest.mark.parametrize("alg", ["default", "coll_pipeline", "p2p_pipeline"])
@pytest.mark.parametrize("streams", [2, 3])
def test_columnwise_copy_streams(d, alg, streams):
    """memcpy pulls split over several copy streams (engines) per peer, joined per block."""
    cfg = AlgoConfig(algorithm=alg, backend="ipc", s=2, copy_streams=streams)
    plan, _ = build_tp_columnwise(0, d, 16 * d, 8, 12, DT_F32, DT_F32, cfg)
    assert plan.nstreams == 2 + (d - 1) * streams
    _run_col(d, m=16 * d, n=8, k=12, cfg=cfg)


@pytest.mark.parametrize("d", [2, 3, 4])
@pytest.mark.parametrize("sig", [SIG_STREAM, SIG_KERNEL])
def test_in_kernel_allgather_plan(d, sig):
    """coll_pipeline fused with CU copies = ONE launch whose copy workgroups pull every peer's
    blocks after its READY and ACK it; the GEMM tiles gate on the blocks' ARRIVE flags."""
    cfg = AlgoConfig(algorithm="coll_pipeline", backend="ipc", fused=True, s=2, signal=sig,
                     protocol="kernel", copy_blocks=16)
    _run_col(d, m=256 * d, n=256, k=64, cfg=cfg, epochs=3)
    plan, _ = build_tp_columnwise(0, d, 256 * d, 256, 64, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == 1 and g[0].args["ag"]["ctas"] == 16 and g[0].args["tile"] == 19
    assert not any(op.kind in (OP_COPY, OP_COPY_MULTI) for op in plan.ops)
    assert max(op.stream for op in plan.ops) == 0  # everything on the caller's stream
    with pytest.raises(ValueError):  # the persistent 256x256 kernel carries the copies
        build_tp_columnwise(0, d, 16 * d, 8, 8, DT_F32, DT_F32, cfg)


def test_in_kernel_allgather_ack_protocol_negative():
    """Without the READY signals the copy workgroups can never start: a deadlock."""
    from ddlb_amd.parallel.sim import Deadlock

    cfg = AlgoConfig(algorithm="coll_pipeline", backend="ipc", fused=True, s=2,
                     protocol="kernel", copy_blocks=8)
    built = [build_tp_columnwise(r, 2, 512, 256, 64, DT_F32, DT_F32, cfg) for r in range(2)]
    plans = [p for p, _ in built]
    for p in plans:  # drop READY: the copy workgroups can never start
        p.ops = [op for op in p.ops if not (op.kind == OP_SIGNAL and any(
            f.buf == "flags" and f.owner is not None for f in op.args["flags"]))]
    sim = Simulator(plans, make_buffers(plans))
    with pytest.raises(Deadlock):
        sim.run_epoch()


def test_in_kernel_allgather_shape_rules():
    """The gated persistent pt4 kernel that carries the in-kernel all-gather unrolls its tile body
    by LDS-buffer parity (an even number of 128-byte K-tiles) and has no fused activation: the
    plan builder refuses other configs instead of failing in the launch."""
    cfg = AlgoConfig(algorithm="coll_pipeline", backend="ipc", fused=True, s=2, protocol="kernel",
                     copy_blocks=8)
    build_tp_columnwise(0, 2, 512, 256, 64, DT_F32, DT_F32, cfg)  # 2 K-tiles of f32
    with pytest.raises(ValueError, match="even number"):
        build_tp_columnwise(0, 2, 512, 256, 96, DT_F32, DT_F32, cfg)  # 3 K-tiles
    act = AlgoConfig(algorithm="coll_pipeline", backend="ipc", fused=True, s=2, protocol="kernel",
                     copy_blocks=8, act=1)
    with pytest.raises(ValueError, match="activation"):
        build_tp_columnwise(0, 2, 512, 256, 64, DT_F32, DT_F32, act)


@pytest.mark.parametrize("alg,fused,proto", [("coll_pipeline", False, "memcpy"),
                                             ("coll_pipeline", True, "memcpy"),
                                             ("coll_pipeline", True, "kernel"),
                                             ("p2p_pipeline", True, "memcpy")])
@pytest.mark.parametrize("backend", ["rccl", "ipc"])
def test_cu_split_reserves_every_gemm(alg, fused, proto, backend):
    """with comm_cus > 0 EVERY compute-stream GEMM (gated, in-kernel all-gather and
    plain) leaves at least comm_cus CUs: its persistent grid fits the masked compute stream."""
    if backend == "rccl" and proto == "kernel":
        pytest.skip("kernel copies are an ipc protocol")
    cfg = AlgoConfig(algorithm=alg, backend=backend, fused=fused, protocol=proto, s=2,
                     comm_cus=48, copy_blocks=8)
    plan, _ = build_tp_columnwise(0, 2, 1024, 256, 64, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM and op.stream == 0]
    assert g and all(op.args["reserve_cus"] >= 48 for op in g)


@pytest.mark.parametrize("queues,first", [("4", True), ("1", False)])
def test_rccl_fused_gemm_enqueued_first(monkeypatch, queues, first):
    """The RCCL-fed gated GEMM goes ahead of its collectives (its own tiles start at once) when
    the process has >= 2 hardware queues; with one in-order queue it stays last (its spinning
    tiles would otherwise sit in front of the collectives that set their flags)."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", queues)
    for alg in ("coll_pipeline", "p2p_pipeline"):
        cfg = AlgoConfig(algorithm=alg, backend="rccl", fused=True, s=2)
        plan, _ = build_tp_columnwise(0, 4, 64, 8, 8, DT_F32, DT_F32, cfg)
        kinds = [op.kind for op in plan.ops]
        assert (kinds[0] == OP_GEMM) == first and (kinds[-1] == OP_GEMM) == (not first)
        _run_col(4, m=64, n=8, k=8, cfg=cfg, epochs=2)


@pytest.mark.parametrize("side", [False, True])
@pytest.mark.parametrize("alg", ["coll_pipeline", "p2p_pipeline"])
def test_rccl_fused_signal_stream(alg, side):
    """``sig_side=False`` (default): the stage signal kernels follow their collective on the comm
    stream (no event hand-off); True: on a third stream behind one event per stage. Same result,
    race-free either way."""
    cfg = AlgoConfig(algorithm=alg, backend="rccl", fused=True, s=2, sig_side=side)
    _run_col(4, m=64, n=8, k=8, cfg=cfg, epochs=2)
    plan, _ = build_tp_columnwise(0, 4, 64, 8, 8, DT_F32, DT_F32, cfg)
    assert all(op.stream == (2 if side else S_COMM) for op in plan.ops if op.kind == OP_SIGNAL)
    assert any(op.kind in (OP_RECORD, OP_WAIT) for op in plan.ops) == side


@pytest.mark.parametrize("d,be", [(1, "rccl"), (2, "rccl"), (2, "ipc"), (4, "rccl"), (4, "ipc")])
def test_split_k_full_gemm(d, be):
    """A full GEMM whose 256x256 grid covers few CUs and whose K is long runs K-split: ONE
    persistent launch over (slice, tile) pairs writing S partials, summed by one reduce op; exact
    result, race-free."""
    m, n, k = 256 * d, 256, 2048
    cfg = AlgoConfig(algorithm="default", backend=be)
    plan, _ = build_tp_columnwise(0, d, m, n, k, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == 1 and g[0].stream == 0 and g[0].args["ksplit"] == 4
    assert g[0].args["K"] == k // 4 and g[0].args["lda"] == k and g[0].args["tile"] == 19
    assert sum(op.kind == OP_REDUCE for op in plan.ops) == 1
    _run_col(d, m, n, k, cfg, epochs=2)


def test_split_k_not_for_full_machine_or_short_k():
    """The flagship (1024 tiles), a short K, an explicit tile and a fused activation keep one
    unsplit GEMM; BASELINE config #2's full GEMM (128 tiles, K = 8192) splits in two."""
    for (m, n, k, kw) in [(65536, 1024, 1024, {}), (8192, 1024, 1024, {}),
                          (8192, 1024, 8192, dict(tile=18)), (8192, 1024, 8192, dict(act=1))]:
        cfg = AlgoConfig(algorithm="default", backend="rccl", **kw)
        plan, _ = build_tp_columnwise(0, 1, m, n, k, DT_BF16, DT_BF16, cfg)
        g = [op for op in plan.ops if op.kind == OP_GEMM]
        assert len(g) == 1 and g[0].args["ksplit"] == 1, (m, n, k, kw)
    plan, _ = build_tp_columnwise(0, 1, 8192, 1024, 8192, DT_BF16, DT_BF16,
                                  AlgoConfig(algorithm="default", backend="rccl"))
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == 1 and g[0].args["ksplit"] == 2


def test_ksplit_rejects_tables_and_flags():
    from ddlb_amd.parallel.plan import Plan, Ref

    plan = Plan(0, 1)
    a = plan.buffer("a", 1 << 20)
    with pytest.raises(ValueError):
        plan.gemm(0, a, a, a, M=256, N=256, K=256, lda=512, ldb=512, ldc=256, din=DT_F32,
                  dout=DT_F32, ksplit=2, flags=Ref("a", 0))
    with pytest.raises(ValueError):
        plan.gemm(0, a, a, a, M=256, N=256, K=256, lda=512, ldb=512, ldc=256, din=DT_F32,
                  dout=DT_F32, ksplit=2, a_grp=128, a_gstride=256)


@pytest.mark.parametrize("be", ["rccl", "ipc"])
def test_split_k_p2p_shard_gemms(be):
    """p2p_pipeline's per-shard GEMMs (plain C rows) take the K-split too when each shard has
    few tiles and K is long (BASELINE 4b: m = 65536, k = 8192 at d = 8); one scratch buffer is
    reused on stream 0 between shards, race-free."""
    d, m, n, k = 2, 512, 256, 2048
    cfg = AlgoConfig(algorithm="p2p_pipeline", backend=be)
    plan, _ = build_tp_columnwise(0, d, m, n, k, DT_F32, DT_F32, cfg)
    g = [op for op in plan.ops if op.kind == OP_GEMM]
    assert len(g) == d and all(op.args["ksplit"] == 4 for op in g)
    assert sum(op.kind == OP_REDUCE for op in plan.ops) == d
    _run_col(d, m, n, k, cfg, epochs=2)


def test_split_k_factor_rule():
    """The K-split rule (ops.gemm.split_k_factor): S slices only while S x tiles fit the CUs and
    every slice keeps >= 16 K-tiles of an even count; a compute partition's fewer CUs split less."""
    from ddlb_amd.ops.gemm import split_k_factor as f

    assert f(8192, 1024, 8192, 2, 256) == 2          # BASELINE config #2: 128 tiles
    assert f(2048, 1024, 8192, 2, 256) == 4          # 32 tiles
    assert f(2048, 1024, 8192, 1, 256) == 4          # fp8: 64 K-tiles of 128 B
    assert f(65536, 1024, 1024, 2, 256) == 1         # the flagship fills the chip
    assert f(8192, 1024, 1024, 2, 256) == 1          # short K: 8 K-tiles per slice is too few
    assert f(8192, 1024, 8192, 2, 32) == 1           # a 32-CU partition: 128 tiles already fill it
    assert f(1000, 1024, 8192, 2, 256) == 1          # ragged M


def test_gate_reserve_floor():
    """A gated GEMM fed by other kernels never leaves fewer than 32 CUs free (smaller reserves
    hung the emulated RCCL-fed plan, profiles/r04/r4_33_*); larger requests pass through."""
    for alg, be in [("coll_pipeline", "rccl"), ("p2p_pipeline", "rccl"), ("coll_pipeline", "ipc"),
                    ("p2p_pipeline", "ipc")]:
        for req, want in [(0, 32), (16, 32), (48, 48)]:
            cfg = AlgoConfig(algorithm=alg, backend=be, fused=True, s=2, reserve_cus=req)
            plan, _ = build_tp_columnwise(0, 4, 64, 8, 8, DT_F32, DT_F32, cfg)
            g = [op for op in plan.ops if op.kind == OP_GEMM and op.args["flags"] is not None]
            assert g and all(op.args["reserve_cus"] == want for op in g), (alg, be, req)


@pytest.mark.parametrize("alg,s", [("coll_pipeline", 2), ("coll_pipeline", 4), ("p2p_pipeline", 1)])
@pytest.mark.parametrize("reserve", [0, 32, 48])
def test_rccl_fed_gate_caps_the_communicator(alg, s, reserve):
    """The RCCL-fed gated GEMM's communicator launches at most reserve_cus workgroups: the plan
    records the cap, the binder's check derives it (GEMM grid + RCCL grid <= num_cus by
    construction) and refuses a plan whose cap is missing or above the reserve."""
    import copy

    from ddlb_amd.parallel.context import rccl_gate_cap

    cfg = AlgoConfig(algorithm=alg, backend="rccl", fused=True, s=s, reserve_cus=reserve)
    for d in (2, 8):
        plan, _ = build_tp_columnwise(1, d, 512 * d, 256, 256, DT_F32, DT_F32, cfg)
        want = max(reserve, 32)
        assert plan.meta["rccl_max_ctas"] == want
        assert rccl_gate_cap(plan) == want
        for bad in (0, want + 1):
            p2 = copy.copy(plan)
            p2.meta = dict(plan.meta, rccl_max_ctas=bad)
            with pytest.raises(ValueError, match="CTA cap"):
                rccl_gate_cap(p2)
    # a CU split keeps RCCL's default (the collectives own their CUs)
    cm = AlgoConfig(algorithm=alg, backend="rccl", fused=True, s=s, comm_cus=32)
    plan, _ = build_tp_columnwise(0, 4, 2048, 256, 256, DT_F32, DT_F32, cm)
    assert plan.meta["rccl_max_ctas"] == 0 and rccl_gate_cap(plan) == 0
    # plans without a gated GEMM fed by RCCL need no cap
    for c in (AlgoConfig(algorithm=alg, backend="rccl", s=s),
              AlgoConfig(algorithm=alg, backend="ipc", fused=True, s=s)):
        plan, _ = build_tp_columnwise(0, 4, 2048, 256, 256, DT_F32, DT_F32, c)
        assert rccl_gate_cap(plan) == 0


def test_rccl_fed_p2p_reads_a_through_a_table():
    """the p2p RCCL-fed gated GEMM's own shard is never gated only in the
    table-A kernel; the plan gives it a row-block table and never raises ARRIVE[rank]."""
    d, m = 4, 4096
    cfg = AlgoConfig(algorithm="p2p_pipeline", backend="rccl", fused=True)
    for r in range(d):
        plan, _ = build_tp_columnwise(r, d, m, 256, 256, DT_F32, DT_F32, cfg)
        g = [op for op in plan.ops if op.kind == OP_GEMM]
        assert len(g) == 1 and g[0].args["tile_order"] == 3 and g[0].args["first_shard"] == r
        assert g[0].args["shard_rows"] == m // d and len(g[0].args["a_shards"]) == d
        raised = [ref for op in plan.ops if op.kind == OP_SIGNAL for ref in op.args["flags"]]
        assert raised and all(ref.off != 4 * (2 * d + 2 * d + r) for ref in raised)


def test_gemm_first_only_on_separate_queues(monkeypatch):
    """the gated GEMM goes ahead of its producers only when its stream (normal
    priority) and theirs (high priority: another hardware-queue pool) cannot share a queue."""
    cfg = AlgoConfig(algorithm="coll_pipeline", backend="rccl", fused=True, s=2)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    plan, _ = build_tp_columnwise(0, 2, 2048, 256, 256, DT_F32, DT_F32, cfg)
    assert plan.meta["gemm_first"] and plan.ops[0].kind == OP_GEMM
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")
    plan, _ = build_tp_columnwise(0, 2, 2048, 256, 256, DT_F32, DT_F32, cfg)
    assert not plan.meta["gemm_first"] and plan.ops[-1].kind == OP_GEMM
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    off = AlgoConfig(algorithm="p2p_pipeline", backend="rccl", fused=True, gemm_first=False)
    plan, _ = build_tp_columnwise(0, 2, 2048, 256, 256, DT_F32, DT_F32, off)
    assert not plan.meta["gemm_first"] and plan.ops[-1].kind == OP_GEMM
