"""The one-GPU per-rank budget emulation (ddlb_amd.parallel.budget, scripts/plan_budget.py): every
N>1 bench candidate's rank plan, rewritten to one rank, must be a valid plan (no peer refs, no
RCCL calls) that runs to completion with its flags pre-set, keep every GEMM of the original, and
move the same bytes as the original's transfers."""

import math
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from ddlb_amd.parallel.algorithms import build_tp_columnwise, build_tp_rowwise  # noqa: E402
from ddlb_amd.parallel.budget import (PRESET, emulate, flag_buffers, gemm_only,  # noqa: E402
                                      op_counts)
from ddlb_amd.parallel.plan import DT_F32, OP_GEMM, RCCL_OPS  # noqa: E402
from ddlb_amd.parallel.sim import Simulator, make_buffers  # noqa: E402


def _cfgs():
    from plan_budget import candidate_cfgs

    out = []
    for prim in ("tp_columnwise", "tp_rowwise"):
        for label, _, cfg in candidate_cfgs(prim, "bfloat16", 8):
            out.append((prim, label, cfg))
    return out


def _shape(prim, cfg, d):
    s = cfg.s if cfg.algorithm == "coll_pipeline" else 1
    if prim == "tp_columnwise" and cfg.fused and cfg.protocol == "kernel":
        return 256 * d * s // math.gcd(256, d * s), 256, 64
    if prim == "tp_columnwise":
        return 4 * d * s, 8, 12
    return 4 * d * s, 8, 4 * d


@pytest.mark.parametrize("d", [2, 8])
@pytest.mark.parametrize("prim,label,cfg", _cfgs(), ids=[c[1] for c in _cfgs()])
def test_emulated_plan_runs_alone(d, prim, label, cfg):
    m, n, k = _shape(prim, cfg, d)
    build = build_tp_columnwise if prim == "tp_columnwise" else build_tp_rowwise
    plan, _ = build(0, d, m, n, k, DT_F32, DT_F32, cfg)
    ep = emulate(plan)
    assert ep.world == 1 and not any(op.kind in RCCL_OPS for op in ep.ops)
    assert not any(s.symmetric for s in ep.buffers.values())
    for op in ep.ops:  # no ref to a peer's copy is left
        for v in op.args.values():
            refs = v if isinstance(v, list) else [v]
            for r in refs:
                assert getattr(r, "owner", None) is None
    assert op_counts(ep).get("gemm", 0) == op_counts(plan).get("gemm", 0)
    for p in (ep, gemm_only(ep)):
        bufs = make_buffers([p])
        for name in flag_buffers(p):
            bufs[0][name].view(torch.int32).fill_(PRESET)
        sim = Simulator([p], bufs, check_races=False)  # pre-set flags drop the ordering
        for _ in range(2):
            sim.run_epoch()
    g = gemm_only(ep)
    assert all(op.kind == OP_GEMM and op.stream == 0 and op.args["flags"] is None
               for op in g.ops)


def test_link_bytes_model():
    """The per-peer link model: an all-gather of a rank's m/d rows moves them to every peer; the
    in-kernel all-gather and the direct-access GEMM move the same bytes; a direct-store GEMM
    writes each peer's output block."""
    from ddlb_amd.parallel.algorithms import AlgoConfig
    from ddlb_amd.parallel.budget import link_bytes
    from ddlb_amd.parallel.plan import DT_BF16

    d, m, n, k = 8, 65536, 1024, 1024
    shard = m // d * k * 2
    for cfg in (AlgoConfig(algorithm="default", backend="rccl"),
                AlgoConfig(algorithm="coll_pipeline", backend="rccl", s=8, fused=True),
                AlgoConfig(algorithm="direct", backend="ipc"),
                AlgoConfig(algorithm="coll_pipeline", backend="ipc", fused=True, s=4,
                           protocol="kernel", copy_blocks=32),
                AlgoConfig(algorithm="coll_pipeline", backend="ipc", s=4)):
        plan, _ = build_tp_columnwise(3, d, m, n, k, DT_BF16, DT_BF16, cfg)
        lb = link_bytes(plan)
        assert sorted(lb) == [p for p in range(d) if p != 3]
        assert all(v == shard for v in lb.values()), (cfg, lb)
    plan, _ = build_tp_rowwise(0, d, 16384, 8192, 8192, DT_BF16, DT_BF16,
                               AlgoConfig(algorithm="p2p_pipeline", backend="ipc", fused=True))
    assert all(v == 16384 // d * 8192 * 2 for v in link_bytes(plan).values())


def test_emulated_rccl_stand_in_respects_the_cta_cap():
    """The copy kernels standing in for RCCL in the one-GPU budget never exceed the plan's RCCL
    CTA cap (the RCCL-fed gated GEMM's reserve), whatever --rccl-blocks asks for."""
    from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise
    from ddlb_amd.parallel.budget import emulate
    from ddlb_amd.parallel.plan import DT_BF16, OP_COPY

    cfg = AlgoConfig(algorithm="coll_pipeline", backend="rccl", fused=True, s=4)
    plan, _ = build_tp_columnwise(0, 8, 65536, 1024, 1024, DT_BF16, DT_BF16, cfg)
    assert plan.meta["rccl_max_ctas"] == 32
    for ask, want in [(6, 6), (32, 32), (64, 32)]:
        ep = emulate(plan, rccl_blocks=ask)
        blocks = {op.args["max_blocks"] for op in ep.ops if op.kind == OP_COPY}
        assert blocks == {want}, (ask, blocks)
