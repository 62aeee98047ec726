"""Multi-GPU preflight plans on the CPU simulator (d simulated ranks, byte-exact, race-checked):
the checks bench.py runs before an N>1 job must themselves be correct and deadlock-free, or a
healthy node would be reported broken."""

import pytest
import torch

from ddlb_amd.parallel import preflight as pf
from ddlb_amd.parallel.sim import Simulator, make_buffers

NB = 4096


@pytest.mark.parametrize("d", [2, 3, 4, 8])
@pytest.mark.parametrize("phase", [p for p in pf.IPC_PHASES if p not in pf.PRIMITIVE_PHASES])
def test_ipc_plan_moves_every_peers_pattern(d, phase):
    plans = [pf.build_ipc_plan(r, d, phase, NB) for r in range(d)]
    bufs = make_buffers(plans)
    sim = Simulator(plans, bufs, check_races=True)
    for ep in (1, 2):
        for r in range(d):
            bufs[r]["X"].view(torch.int32)[:] = pf.pattern(r, NB, ep)
            bufs[r]["R"].view(torch.int32).fill_(-1)
        sim.run_epoch()
        if phase in ("ipc_kernel", "ipc_sdma", "ipc_push", "ipc_batch"):
            for r in range(d):
                rv = bufs[r]["R"].view(torch.int32)
                for p in range(d):
                    if p != r:
                        assert torch.equal(rv[p * NB // 4:(p + 1) * NB // 4],
                                           pf.pattern(p, NB, ep)), (r, p, ep)
        # every flag word ends at this epoch: the handshakes completed
        for r in range(d):
            flags = bufs[r]["flags"].view(torch.int32)
            assert int(flags[d:2 * d].sum()) == ep * (d - 1)  # ACKs from every peer


def test_pattern_differs_per_owner_and_epoch():
    a, b, c = pf.pattern(0, NB, 1), pf.pattern(1, NB, 1), pf.pattern(0, NB, 2)
    assert not torch.equal(a, b) and not torch.equal(a, c)
    assert int((a == b).sum()) == 0


@pytest.mark.parametrize("d", [2, 4, 8])
def test_rccl_plan(d):
    plans = [pf.build_rccl_plan(r, d, NB, 256) for r in range(d)]
    bufs = make_buffers(plans)
    for r in range(d):
        bufs[r]["SEND"].view(torch.int32)[:] = pf.pattern(r, NB, 1)
        bufs[r]["RSIN"].view(torch.float32)[:] = pf.rs_input(r, d, 256)
    Simulator(plans, bufs, check_races=True).run_epoch()
    for r in range(d):
        ag = bufs[r]["AG"].view(torch.int32)
        for q in range(d):
            assert torch.equal(ag[q * NB // 4:(q + 1) * NB // 4], pf.pattern(q, NB, 1))
        assert torch.equal(bufs[r]["RSOUT"].view(torch.float32), pf.rs_expected(r, d, 256))


def test_needs_maps_candidates_to_checks():
    assert pf.needs("pytorch", {}) == ["torch_nccl"]
    assert pf.needs("native", {"backend": "rccl"}) == ["rccl"]
    assert pf.needs("native", {"backend": "rccl", "fused": True}) == ["rccl", "rccl_cap",
                                                                     "rccl_fused"]
    assert pf.needs("native", {"backend": "rccl", "fused": True, "comm_cus": 32}) == \
        ["rccl", "rccl_fused_cm"]
    assert pf.needs("native", {"backend": "ipc", "multicast_protocol": "memcpy",
                               "graph": False}) == ["ipc", "ipc_sdma"]
    # no "graph" key = the option default "auto": graph replay signals with the kernels
    assert pf.needs("native", {"backend": "ipc", "multicast_protocol": "memcpy"}) == \
        ["ipc", "ipc_ksig", "ipc_sdma"]
    agk = pf.needs("native", {"backend": "ipc", "multicast_protocol": "kernel", "fused": True,
                              "algorithm": "coll_pipeline", "graph": True})
    assert agk == ["ipc", "ipc_ksig", "ipc_kernel", "ipc_agk"]
    dstore = pf.needs("native", {"backend": "ipc", "algorithm": "p2p_pipeline", "fused": True,
                                 "graph": False}, primitive="tp_rowwise")
    assert dstore == ["ipc", "ipc_ksig", "ipc_sdma", "ipc_dstore"]
    assert "ipc_kernel" in pf.needs("native", {"backend": "ipc", "algorithm": "direct"})
    assert "ipc_push" in pf.needs("native", {"backend": "ipc", "direction": "push"})
    assert pf.needs("native", {"backend": "ipc", "multicast_protocol": "batch_memcpy",
                               "graph": False}) == ["ipc", "ipc_batch"]
    assert pf.needs("compute_only", {}) == []


def test_merge_over_ranks():
    per_rank = [{"ipc": "ok (3 ms)", "ipc_sdma": "ok"},
                {"ipc": "ok (4 ms)", "ipc_sdma": "failed: AssertionError: 3 words differ"},
                {"ipc": "ok (2 ms)"}]
    m = pf.merge(per_rank, ("ipc", "ipc_sdma", "ipc_kernel"))
    assert m["ipc"].startswith("ok")
    assert m["ipc_sdma"].startswith("failed: AssertionError")
    assert m["ipc_kernel"] == "failed: timeout"


@pytest.mark.parametrize("d", [2, 3, 4, 8])
@pytest.mark.parametrize("phase", sorted(pf.PRIMITIVE_PHASES))
def test_primitive_phases_simulate(d, phase):
    """The primitive-level phases (in-kernel AG, direct store, RCCL-fed gated GEMM) at their
    preflight shape: the real plan builders, simulated for d ranks, exact."""
    from ddlb_amd.parallel.algorithms import build_tp_columnwise, build_tp_rowwise
    from ddlb_amd.parallel.plan import DT_F32
    from ddlb_amd.primitives.native_common import algo_config
    from ddlb_amd.primitives.registry import resolve

    prim, opts = pf.PRIMITIVE_PHASES[phase]
    m, n, k = pf.primitive_shape(d)
    cls, o, _ = resolve(prim, "native", dict(opts))
    merged = {**cls.DEFAULT_OPTIONS, **o}
    for key, alias in cls.OPTION_ALIASES.items():
        merged[key] = alias.get(merged[key], merged[key])
    cfg = algo_config(merged)
    build = build_tp_columnwise if prim == "tp_columnwise" else build_tp_rowwise
    for r in range(d):  # the shape passes every builder check at every rank
        build(r, d, m, n, k, DT_F32, DT_F32, cfg)
        if phase in pf.PRIMITIVE_SHAPES:  # the phase's own (larger, CU-filling) shape too
            build(r, d, *pf.PRIMITIVE_SHAPES[phase](d), DT_F32, DT_F32, cfg)
    from test_plans_sim import _run_col, _run_row

    (_run_col if prim == "tp_columnwise" else _run_row)(d, m, n, k, cfg, epochs=2)


@pytest.mark.parametrize("family,phases", [("rccl", pf.RCCL_PHASES), ("ipc", pf.IPC_PHASES)])
def test_every_declared_phase_has_a_check(family, phases):
    """A declared phase without a check would be reported 'failed: timeout' on every node and
    silently drop the candidates that need it (rccl_fused_cm)."""
    assert sorted(pf.phase_checks(None, family)) == sorted(phases)


def test_run_checks_report_every_phase(monkeypatch):
    """Both families, native layer stubbed: every phase ends with its own status (ok or the
    check's own error), in order, and 'failed: timeout' can only come from a killed child."""

    class FakeComm:
        rank, world_size, device = 0, 2, "cpu"

        def native(self):
            raise RuntimeError("no native layer in this test")

        def barrier(self):
            pass

    ran = []

    def fake_primitive(comm, phase, epochs=2):
        ran.append(phase)
        if phase == "rccl_fused":
            raise TimeoutError("stand-in for RCCL's own error")

    monkeypatch.setattr(pf, "run_primitive_check", fake_primitive)
    monkeypatch.setattr(pf, "_torch_nccl_check", lambda comm: None)
    res = pf.run_rccl_checks(FakeComm())
    assert list(res) == list(pf.RCCL_PHASES)
    assert res["torch_nccl"].startswith("ok")
    assert res["rccl"].startswith("failed: RuntimeError: no native layer")
    assert res["rccl_cap"].startswith("failed: RuntimeError: no native layer")
    assert res["rccl_fused"].startswith("failed: TimeoutError: stand-in")
    assert res["rccl_fused_cm"].startswith("ok")
    assert "rccl_fused_cm" in ran
    res = pf.run_ipc_checks(FakeComm())
    assert list(res) == list(pf.IPC_PHASES)
    for ph in pf.IPC_PHASES:
        want = "ok" if ph in pf.PRIMITIVE_PHASES else "failed: RuntimeError"
        assert res[ph].startswith(want), (ph, res[ph])
        assert res[ph] != "failed: timeout"
    merged = pf.merge([res, res], pf.IPC_PHASES)
    assert not any(v == "failed: timeout" for v in merged.values())


class _FakeHolder:
    """cap_probe's holder: ``resident`` workgroups become resident (of those started)."""

    def __init__(self, resident=None, timeout_bits=0):
        self.resident, self.bits = resident, timeout_bits
        self.n, self.released, self.events = 0, False, []

    def start(self, n):
        self.n = n
        self.events.append(("start", n))

    def arrived(self):
        return self.n if self.resident is None else min(self.resident, self.n)

    def release(self):
        self.released = True
        self.events.append(("release",))

    def timeout_bits(self):
        return self.bits


class _Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t

    def sleep(self, dt):
        self.t += dt


@pytest.mark.parametrize("finish_after", [0.0, 0.05])
def test_cap_probe_observes_capped_collective(finish_after):
    """rccl_cap: num_cus - cap CUs held, barrier, then the capped all-gather
    must finish while they are held; the holders are released afterwards, in every case."""
    clk, h, order = _Clock(), _FakeHolder(), []
    t_launch = []

    def launch():
        order.append("launch")
        t_launch.append(clk.t)

    res = pf.cap_probe(h, launch, lambda: clk.t - t_launch[0] >= finish_after,
                       lambda: order.append("barrier"), ncu=256, cap=32, sleep=clk.sleep,
                       clock=clk)
    assert h.events[0] == ("start", 224) and h.released
    assert order == ["barrier", "launch"]
    assert res["held_cus"] == 224 and res["cap"] == 32
    assert res["held_ms"] >= finish_after * 1e3 - 1e-6


def test_cap_probe_refuses_collective_that_cannot_finish():
    """The refusal path: a collective that never completes beside the held CUs (RCCL launched
    more workgroups than the cap, or needs CUs the holders took) fails the phase after the bound
    -- not a hang: the holders are released, so the collective drains afterwards."""
    clk, h = _Clock(), _FakeHolder()
    with pytest.raises(RuntimeError, match="did not finish .* beside 224 held CUs"):
        pf.cap_probe(h, lambda: None, lambda: False, lambda: None, ncu=256, cap=32,
                     finish_s=5.0, sleep=clk.sleep, clock=clk)
    assert h.released and 5.0 <= clk.t < 5.1


def test_cap_probe_holders_not_resident_and_spin_bound():
    clk = _Clock()
    h = _FakeHolder(resident=200)
    with pytest.raises(RuntimeError, match="only 200 of 224 holder workgroups"):
        pf.cap_probe(h, lambda: None, lambda: True, lambda: None, ncu=256, cap=32,
                     sleep=clk.sleep, clock=clk)
    assert h.released
    h = _FakeHolder(timeout_bits=4)
    with pytest.raises(RuntimeError, match="bounded spin gave up"):
        pf.cap_probe(h, lambda: None, lambda: True, lambda: None, ncu=256, cap=32,
                     sleep=clk.sleep, clock=clk)
    with pytest.raises(ValueError):
        pf.cap_probe(_FakeHolder(), lambda: None, lambda: True, lambda: None, ncu=32, cap=32)


def test_fused_rccl_cap_is_the_gate_reserve():
    """The cap the probe checks is the one the fused candidates bind (one CU per shader array)."""
    for d in (2, 4, 8):
        assert pf.fused_rccl_cap(d) == 32
