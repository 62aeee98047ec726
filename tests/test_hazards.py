"""The simulator's checker must catch broken schedules (negative tests), not only pass good ones."""

import pytest

from ddlb_amd.parallel.plan import DT_F32, SIG_STREAM, Plan
from ddlb_amd.parallel.sim import Deadlock, RaceDetected, Simulator, make_buffers


def _two_rank(builder):
    plans = [builder(r) for r in range(2)]
    return Simulator(plans, make_buffers(plans))


def test_missing_event_edge_is_a_race():
    def build(r):
        p = Plan(r, 2, nstreams=2)
        x = p.buffer("X", 64)
        y = p.buffer("Y", 64)
        p.memset(1, x, 64, 1)          # producer on stream 1
        p.copy(0, y, x, 64)            # consumer on stream 0, no edge
        return p

    with pytest.raises(RaceDetected):
        _two_rank(build).run_epoch()


def test_event_edge_orders_it():
    def build(r):
        p = Plan(r, 2, nstreams=2)
        x = p.buffer("X", 64)
        y = p.buffer("Y", 64)
        p.memset(1, x, 64, 1)
        p.edge(1, 0)
        p.copy(0, y, x, 64)
        return p

    sim = _two_rank(build)
    sim.run_epoch()
    assert int(sim.bufs[0]["Y"][0]) == 1


def test_remote_read_without_signal_is_a_race():
    def build(r):
        p = Plan(r, 2, nstreams=2)
        x = p.buffer("X", 64, symmetric=True)
        y = p.buffer("Y", 64)
        p.buffer("flags", 256, symmetric=True, zero=True)
        p.memset(0, x, 64, r + 1)                    # write my shard
        p.copy(1, y, x.at(1 - r), 64)                # pull the peer's, unsynchronised
        return p

    with pytest.raises(RaceDetected):
        _two_rank(build).run_epoch()


def test_remote_read_with_ready_signal_is_clean():
    from ddlb_amd.parallel.plan import Ref

    def build(r):
        p = Plan(r, 2, nstreams=2)
        x = p.buffer("X", 64, symmetric=True)
        y = p.buffer("Y", 64)
        p.buffer("flags", 256, symmetric=True, zero=True)
        p.wait_signal(0, [Ref("flags", 4, None)], SIG_STREAM, delta=-1)  # peer done reading
        p.memset(0, x, 64, r + 1)
        p.signal(0, [Ref("flags", 0, 1 - r)], SIG_STREAM)                 # READY -> peer
        p.wait_signal(1, [Ref("flags", 0, None)], SIG_STREAM)
        p.copy(1, y, x.at(1 - r), 64)
        p.signal(1, [Ref("flags", 4, 1 - r)], SIG_STREAM)                 # ACK -> peer
        return p

    sim = _two_rank(build)
    for _ in range(3):
        sim.run_epoch()
    assert int(sim.bufs[0]["Y"][0]) == 2 and int(sim.bufs[1]["Y"][0]) == 1


def test_missing_ack_makes_next_epoch_racy():
    from ddlb_amd.parallel.plan import Ref

    def build(r):
        p = Plan(r, 2, nstreams=2)
        x = p.buffer("X", 64, symmetric=True)
        y = p.buffer("Y", 64)
        p.buffer("flags", 256, symmetric=True, zero=True)
        p.memset(0, x, 64, r + 1)                    # overwrites while the peer may still read
        p.signal(0, [Ref("flags", 0, 1 - r)], SIG_STREAM)
        p.wait_signal(1, [Ref("flags", 0, None)], SIG_STREAM)
        p.copy(1, y, x.at(1 - r), 64)
        return p

    sim = _two_rank(build)
    with pytest.raises(RaceDetected):
        for _ in range(3):
            sim.run_epoch()


def test_deadlock_detected():
    from ddlb_amd.parallel.plan import Ref

    def build(r):
        p = Plan(r, 2, nstreams=1)
        p.buffer("flags", 256, symmetric=True, zero=True)
        p.wait_signal(0, [Ref("flags", 0, None)], SIG_STREAM)   # both wait first ...
        p.signal(0, [Ref("flags", 0, 1 - r)], SIG_STREAM)       # ... then signal: cycle
        return p

    with pytest.raises(Deadlock):
        _two_rank(build).run_epoch()


def test_mismatched_collectives_deadlock():
    def build(r):
        p = Plan(r, 2, nstreams=1)
        b = p.buffer("B", 64)
        if r == 0:
            p.allgather(0, b, p.buffer("R", 128), 16, DT_F32)
        return p

    with pytest.raises(Deadlock):
        _two_rank(build).run_epoch()


def test_explain_cli_simulates(capsys):
    from ddlb_amd.parallel.explain import main

    main(["--primitive", "tp_rowwise", "-d", "4", "-m", "64", "-n", "8", "-k", "16",
          "--algorithm", "p2p_pipeline", "--backend", "ipc", "--dtype", "float32", "--simulate"])
    out = capsys.readouterr().out
    assert "no race, no deadlock, max|err| = 0.0" in out


def _direct_with_producer(drop_ack: bool):
    """Direct-access plans preceded by a producer that rewrites the own shard every run."""
    from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise
    from ddlb_amd.parallel.plan import OP_COPY, OP_WAIT_SIGNAL, Op, Ref

    d, m, n, k = 2, 16, 8, 8
    plans = []
    for r in range(d):
        plan, io = build_tp_columnwise(r, d, m, n, k, DT_F32, DT_F32,
                                       AlgoConfig(algorithm="direct", backend="ipc"))
        nb = (m // d) * k * 4
        plan.buffer("A_in", nb)
        plan.ops.insert(0, Op(OP_COPY, 0, dict(dst=Ref("A_own"), src=Ref("A_in"), nbytes=nb,
                                               method=0, max_blocks=0)))
        if drop_ack:
            last = max(i for i, op in enumerate(plan.ops) if op.kind == OP_WAIT_SIGNAL)
            del plan.ops[last]
        plans.append(plan)
    return Simulator(plans, make_buffers(plans))


def test_direct_access_ack_protects_next_write():
    sim = _direct_with_producer(drop_ack=False)
    for _ in range(3):
        sim.run_epoch()


def test_direct_access_without_ack_is_a_race():
    sim = _direct_with_producer(drop_ack=True)
    with pytest.raises((RaceDetected, Deadlock)):
        for _ in range(3):
            sim.run_epoch()


def test_redundant_back_to_back_signal_is_flagged():
    """Two identical signals in a row on one stream (the copy-paste duplicate ADVICE r2 found in
    the kernel-protocol pull) are rejected by the simulator instead of silently costing a launch
    per run."""
    from ddlb_amd.parallel.plan import Plan, Ref
    from ddlb_amd.parallel.sim import RedundantOp, Simulator, make_buffers

    plan = Plan(0, 1, nstreams=2)
    plan.buffer("flags", 256, symmetric=True, zero=True)
    f = [Ref("flags", 0)]
    plan.signal(1, f)
    plan.signal(0, f)      # another stream: fine
    plan.signal(1, f, delta=1)  # different value: fine
    Simulator([plan], make_buffers([plan]))
    plan.signal(1, f, delta=1)
    with pytest.raises(RedundantOp):
        Simulator([plan], make_buffers([plan]))


def test_no_bench_plan_has_redundant_signals():
    from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise
    from ddlb_amd.parallel.plan import DT_BF16
    from ddlb_amd.parallel.sim import check_redundant

    for proto in ("memcpy", "batch_memcpy", "kernel"):
        for alg in ("default", "coll_pipeline", "p2p_pipeline"):
            for fused in (False, True):
                cfg = AlgoConfig(algorithm=alg, backend="ipc", protocol=proto, s=2, fused=fused)
                try:
                    plan, _ = build_tp_columnwise(0, 4, 2048, 256, 256, DT_BF16, DT_BF16, cfg)
                except ValueError:
                    continue
                check_redundant(plan)


def test_plan_labels_name_stages():
    from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise
    from ddlb_amd.parallel.plan import DT_BF16

    plan, _ = build_tp_columnwise(0, 2, 1024, 64, 64, DT_BF16, DT_BF16,
                                  AlgoConfig(algorithm="coll_pipeline", backend="ipc", s=2))
    labels = plan.labels()
    assert len(labels) == len(plan.ops)
    assert "gemm s0" in labels and "gemm s1" in labels
    assert "copy p1 b0" in labels and "copy p1 b1" in labels
    assert any(x.startswith("wait_signal flags+") for x in labels)
    plan, _ = build_tp_columnwise(0, 2, 1024, 64, 64, DT_BF16, DT_BF16,
                                  AlgoConfig(algorithm="coll_pipeline", backend="rccl", s=2))
    assert {"allgather #0", "allgather #1"} <= set(plan.labels())
