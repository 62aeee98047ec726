"""Impl-spec grammar, value inference, cartesian expansion, JSON normalisation (reference
``ddlb/cli/benchmark.py:14-118``)."""

import pytest

from ddlb_amd.cli.config import (base_impl_name, build_impl_table, generate_config_combinations,
                                 infer_scalar, normalize_benchmark_config, parse_impl_spec,
                                 parse_int_list, parse_value_list)
from ddlb_amd.cli.benchmark import resolve_csv_path


@pytest.mark.parametrize("tok,val", [("true", True), ("False", False), ("8", 8), ("0", 0),
                                     ("-3", -3), ("0.5", 0.5), ("1e3", 1000.0), ("nccl", "nccl"),
                                     ("08", "08"), ("ucc/tl/nccl", "ucc/tl/nccl"),
                                     (" 12 ", 12)])
def test_infer_scalar(tok, val):
    out = infer_scalar(tok)
    assert out == val and type(out) is type(val)


def test_parse_value_list():
    assert parse_value_list("1,2, 3") == [1, 2, 3]
    assert parse_value_list("nccl") == "nccl"
    assert parse_value_list("") == ""
    assert parse_value_list("AG_before,AG_after") == ["AG_before", "AG_after"]


def test_parse_int_list():
    assert parse_int_list("1024,8192") == [1024, 8192]
    assert parse_int_list([1, "2"]) == [1, 2]


def test_parse_impl_spec():
    name, opts = parse_impl_spec("fuser;algorithm=coll_pipeline;s=2,8;backend=nccl;fused")
    assert name == "fuser"
    assert opts == {"algorithm": "coll_pipeline", "s": [2, 8], "backend": "nccl", "fused": True}
    assert parse_impl_spec("pytorch") == ("pytorch", {})
    with pytest.raises(ValueError):
        parse_impl_spec(";;")


def test_cartesian_expansion_within_base_config():
    cfg = {"pytorch": [{"backend": ["nccl", "rccl"], "order": ["AG_before", "AG_after"]}],
           "native": [{"algorithm": "default"}, {"algorithm": "coll_pipeline", "s": [2, 8]}]}
    out = generate_config_combinations(cfg)
    assert len(out["pytorch"]) == 4
    assert {"backend": "rccl", "order": "AG_after"} in out["pytorch"]
    assert out["native"] == [{"algorithm": "default"},
                             {"algorithm": "coll_pipeline", "s": 2},
                             {"algorithm": "coll_pipeline", "s": 8}]
    ids, opts = build_impl_table(out)
    assert ids[:2] == ["pytorch_0", "pytorch_1"] and "native_2" in ids
    assert opts["native_2"] == {"implementation": "native", "algorithm": "coll_pipeline", "s": 8}


def test_base_impl_name():
    assert base_impl_name("compute_only_3") == "compute_only"
    assert base_impl_name("pytorch") == "pytorch"
    assert base_impl_name("transformer_engine_0") == "transformer_engine"


def test_normalize_defaults_and_errors():
    b = normalize_benchmark_config({"benchmark": {"primitive": "tp_rowwise", "m": 64, "n": [8],
                                                  "k": "16", "implementations": {"pytorch": [{}]}}})
    assert b["m"] == [64] and b["k"] == [16] and b["dtype"] == "float32"
    assert b["time_measurement_backend"] == "cpu_clock" and b["barrier_at_each_iteration"]
    with pytest.raises(ValueError):
        normalize_benchmark_config({"benchmark": {"primitive": "allreduce", "m": 1, "n": 1,
                                                  "k": 1, "implementations": {"x": [{}]}}})
    with pytest.raises(ValueError):
        normalize_benchmark_config({"benchmark": {"primitive": "tp_columnwise", "m": 1}})


def test_csv_path():
    assert resolve_csv_path("r/x_{timestamp}.csv", "tp_columnwise", [1], [2], [3], "bf16",
                            stamp="T") == "r/x_T.csv"
    assert resolve_csv_path(None, "tp_rowwise", [8], [2], [4], "float16", stamp="T") == \
        "results/tp_rowwise_8x4x2_float16_T.csv"


def test_reference_json_configs_parse():
    import json
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for name in ("config.json", "config_tp_rowwise.json"):
        with open(os.path.join(root, "scripts", name)) as f:
            b = normalize_benchmark_config(json.load(f))
        assert generate_config_combinations(b["implementations"])
