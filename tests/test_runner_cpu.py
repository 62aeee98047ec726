"""The runner end to end on the CPU: CSV schema, timing modes, isolation, error rows, resume,
and a 2-rank torchrun launch through the CLI (gloo)."""

import csv
import json
import os
import subprocess
import sys

import pytest

from ddlb_amd.utils.stats import CSV_COLUMNS, EXTRA_COLUMNS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ, DDLB_DEVICE="cpu", DDLB_PROGRESS="0", DDLB_TRACEBACK="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "DDLB_CHILD_INIT_METHOD", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def _config(tmp_path, impls, **kw):
    b = {"primitive": "tp_columnwise", "m": 64, "n": 16, "k": 32, "dtype": "float32",
         "validate": True, "num_iterations": 3, "num_warmups": 1, "profile_iterations": 1,
         "output_csv": str(tmp_path / "out_{timestamp}.csv"), "implementations": impls}
    b.update(kw)
    return {"benchmark": b}


def _run_inproc(monkeypatch, config, isolate=False):
    from conftest import free_port

    for k, v in _env().items():
        monkeypatch.setenv(k, v)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "DDLB_CHILD_INIT_METHOD", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("DDLB_MASTER_PORT", str(free_port()))
    from ddlb_amd.cli.benchmark import run_benchmark

    return run_benchmark(config, isolate=isolate)


def _csv_rows(tmp_path):
    files = list(tmp_path.glob("out_*.csv"))
    assert len(files) == 1
    with open(files[0], newline="") as f:
        return list(csv.DictReader(f)), files[0]


@pytest.mark.parametrize("backend,barrier", [("cpu_clock", True), ("cpu_clock", False),
                                             ("cuda_event", True), ("cuda_event", False)])
def test_timing_modes_inprocess(tmp_path, monkeypatch, backend, barrier):
    cfg = _config(tmp_path, {"compute_only": [{"size": ["sharded", "unsharded"]}],
                             "pytorch": [{"order": ["AG_before", "AG_after"],
                                          "empty_cache": False}]},
                  time_measurement_backend=backend, barrier_at_each_iteration=barrier)
    df = _run_inproc(monkeypatch, cfg)
    assert len(df) == 4 and all(df["valid"])
    rows, _ = _csv_rows(tmp_path)
    assert list(rows[0].keys()) == CSV_COLUMNS + EXTRA_COLUMNS + ["spec"]
    for r in rows:
        assert float(r["mean_time (ms)"]) > 0 and r["valid"] == "True"
        assert r["time_measurement_backend"] == backend
    labels = [r["implementation"] for r in rows]
    assert "pytorch (backend=nccl, order=AG_after, empty_cache=False)" in labels
    # TFLOPS formula 2mnk/(t_ms*1e9) per iteration; mean of per-iteration values
    r = rows[0]
    if not barrier:
        t = float(r["mean_time (ms)"])
        assert abs(float(r["Throughput (TFLOPS)"]) - 2 * 64 * 16 * 32 / (t * 1e9)) < 1e-9


def test_isolated_children_error_rows_and_resume(tmp_path, monkeypatch):
    cfg = _config(tmp_path, {"compute_only": [{"size": "unsharded"}],
                             "native": [{"algorithm": "default"}],           # needs a GPU
                             "pytorch": [{"backend": "ucc/tl/ucp"}]},         # rejected backend
                  rowwise=None)
    cfg["benchmark"].pop("rowwise")
    df = _run_inproc(monkeypatch, cfg, isolate=True)
    assert len(df) == 3
    rows, path = _csv_rows(tmp_path)
    by = {json.loads(r["spec"])["implementation"]: r for r in rows}
    assert by["compute_only"]["valid"] == "True" and by["compute_only"]["error"] == ""
    assert by["native"]["valid"] == "False" and "GPU" in by["native"]["error"]
    assert by["pytorch"]["valid"] == "False" and "UCC" in by["pytorch"]["error"]
    # resume: same CSV path, nothing re-run
    cfg["benchmark"]["output_csv"] = str(path)
    cfg["benchmark"]["resume"] = True
    df2 = _run_inproc(monkeypatch, cfg, isolate=False)
    assert len(df2) == 0
    rows2, _ = _csv_rows(tmp_path)
    assert len(rows2) == 3


def test_rowwise_inprocess(tmp_path, monkeypatch):
    cfg = _config(tmp_path, {"compute_only": [{"size": "sharded"}],
                             "pytorch": [{"empty_cache": False}]}, primitive="tp_rowwise")
    df = _run_inproc(monkeypatch, cfg)
    assert len(df) == 2 and all(df["valid"])


def test_cli_torchrun_two_ranks(tmp_path):
    from conftest import free_port

    out = tmp_path / "tr_{timestamp}.csv"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m", "ddlb_amd",
           "--primitive", "tp_rowwise", "-m", "64", "-n", "16", "-k", "32", "--dtype",
           "float32", "--num-iterations", "3", "--num-warmups", "1", "--profile-iterations", "1",
           "--impl", "pytorch;empty_cache=false", "--impl", "compute_only;size=sharded",
           "--output-csv", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    files = list(tmp_path.glob("tr_*.csv"))
    assert len(files) == 1, r.stdout[-3000:]
    with open(files[0], newline="") as f:
        rows = list(csv.DictReader(f))
    assert len(rows) == 2
    for row in rows:
        assert row["world_size"] == "2" and row["valid"] == "True", row


def test_json_script_entry(tmp_path):
    cfg = _config(tmp_path, {"compute_only": [{"size": "unsharded"}]})
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "run_benchmark.py"),
                        str(p)], capture_output=True, text=True, timeout=600, env=_env(),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Benchmark Results" in r.stdout


def test_derived_metrics_undo_the_harness_formula():
    from ddlb_amd.utils.stats import derived_metrics

    m, n, k, d, ms = 4096, 1024, 2048, 4, 2.0
    harness = 2.0 * m * n * k / (ms * 1e9)
    col = derived_metrics("tp_columnwise", "native", "", m, n, k, "bfloat16", d, ms)
    assert col["per_gpu_tflops"] == pytest.approx(harness)
    assert col["algbw_GBps"] == pytest.approx(m * k * 2 / (ms * 1e-3) / 1e9)
    row = derived_metrics("tp_rowwise", "native", "", m, n, k, "bfloat16", d, ms)
    assert row["per_gpu_tflops"] == pytest.approx(harness / d)
    assert row["algbw_GBps"] == pytest.approx(m * n * 2 / (ms * 1e-3) / 1e9)
    sh = derived_metrics("tp_columnwise", "compute_only", "sharded", m, n, k, "float32", d, ms)
    assert sh["per_gpu_tflops"] == pytest.approx(harness / d) and sh["algbw_GBps"] == 0
    assert derived_metrics("tp_columnwise", "native", "", m, n, k, "bfloat16", 1, ms)[
        "algbw_GBps"] == 0
