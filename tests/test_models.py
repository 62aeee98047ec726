"""Model shape catalog (CPU) and the sequence-parallel TP MLP (GPU)."""

import os

import pytest
import torch

from ddlb_amd.models import MODELS, benchmark_configs, layer_gemms


def test_layer_gemms_llama70b_tp8():
    g = {x.name: x for x in layer_gemms("llama3-70b", 8, 8192)}
    assert g["qkv_proj"].as_tuple() == ("tp_columnwise", 8192, (64 + 16) * 128 // 8, 8192)
    assert g["attn_out_proj"].as_tuple() == ("tp_rowwise", 8192, 8192, 8192)
    assert g["mlp_up_proj"].as_tuple() == ("tp_columnwise", 8192, 2 * 28672 // 8, 8192)
    assert g["mlp_down_proj"].as_tuple() == ("tp_rowwise", 8192, 8192, 28672)


@pytest.mark.parametrize("model", sorted(MODELS))
def test_catalog_consistent(model):
    for tp in (1, 2, 4, 8):
        for g in layer_gemms(model, tp, 4096):
            assert g.m == 4096 and g.n > 0 and g.k > 0
    cfgs = benchmark_configs(model, 8, 4096, {"pytorch": [{}]})
    assert len(cfgs) == 4 and all("benchmark" in c for c in cfgs)


def test_models_cli_list(capsys):
    from ddlb_amd.models.__main__ import main

    main(["--model", "gpt3-175b", "--tp", "8", "--tokens", "2048", "--list"])
    out = capsys.readouterr().out
    assert "qkv_proj" in out and "mlp_down_proj" in out


def test_mlp_plans_compose_in_simulator():
    """col(+gelu) output buffer feeds row input: simulate both plan sets for d=2 ranks."""
    from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise, build_tp_rowwise
    from ddlb_amd.parallel.plan import ACT_GELU, DT_F32
    from ddlb_amd.parallel.sim import (Simulator, apply_act, make_buffers, read_tensor,
                                       write_tensor)

    d, S, H, F = 2, 16, 8, 12
    g = torch.Generator().manual_seed(0)
    X = torch.randn(S, H, generator=g)
    W1 = torch.randn(H, F, generator=g)
    W2 = torch.randn(F, H, generator=g)
    ccfg = AlgoConfig(algorithm="coll_pipeline", backend="ipc", s=2, act=ACT_GELU)
    rcfg = AlgoConfig(algorithm="p2p_pipeline", backend="ipc")
    fl, sl = F // d, S // d
    cols = [build_tp_columnwise(r, d, S, fl, H, DT_F32, DT_F32, ccfg) for r in range(d)]
    rows = [build_tp_rowwise(r, d, S, H, F, DT_F32, DT_F32, rcfg) for r in range(d)]
    cb, rb = make_buffers([c[0] for c in cols]), make_buffers([r[0] for r in rows])
    for r in range(d):
        write_tensor(cb[r], cols[r][1].a, X[r * sl:(r + 1) * sl])
        write_tensor(cb[r], cols[r][1].b, W1[:, r * fl:(r + 1) * fl].t().contiguous())
        write_tensor(rb[r], rows[r][1].b, W2[r * fl:(r + 1) * fl].t().contiguous())
    Simulator([c[0] for c in cols], cb).run_epoch()
    for r in range(d):
        write_tensor(rb[r], rows[r][1].a, read_tensor(cb[r], cols[r][1].out).clone())
    Simulator([x[0] for x in rows], rb).run_epoch()
    ref = apply_act(X @ W1, ACT_GELU) @ W2
    for r in range(d):
        torch.testing.assert_close(read_tensor(rb[r], rows[r][1].out), ref[r * sl:(r + 1) * sl],
                                   rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["gelu", "silu"])
def test_sequence_parallel_mlp_world1(act):
    from conftest import free_port

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.models.tp_mlp import SequenceParallelMLP

    os.environ["DDLB_CHILD_INIT_METHOD"] = f"tcp://127.0.0.1:{free_port()}"
    Communicator.reset()
    try:
        mlp = SequenceParallelMLP(hidden=1024, ffn=4096, seq=2048, act=act)
        for _ in range(3):
            out = mlp.forward()
        torch.cuda.synchronize()
        mlp.validate(out)
        mlp.close()
    finally:
        Communicator.reset()
        os.environ.pop("DDLB_CHILD_INIT_METHOD", None)
