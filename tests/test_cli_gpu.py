"""The DDLB-compatible CLI end to end on the GPU: the JSON / CLI config surface expands to every
implementation slot (native algorithms, the reference's fuser / transformer_engine / jax aliases,
pytorch, compute_only), each runs in its own spawned child (fresh HIP context, RCCL control
group), and the CSV has DDLB's columns with every row validated."""

import csv
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ, DDLB_PROGRESS="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "DDLB_CHILD_INIT_METHOD", "LOCAL_WORLD_SIZE", "DDLB_DEVICE"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("primitive", ["tp_columnwise", "tp_rowwise"])
def test_cli_every_slot_world1(tmp_path, primitive):
    from conftest import free_port

    from ddlb_amd.utils.stats import CSV_COLUMNS

    out = tmp_path / "res_{timestamp}.csv"
    impls = ["native;algorithm=default,coll_pipeline,p2p_pipeline;s=2",
             "native;gemm_mode=generic", "fuser;algorithm=coll_pipeline;s=2",
             "transformer_engine", "pytorch;empty_cache=false",
             "compute_only;size=unsharded"]
    if primitive == "tp_columnwise":
        impls += ["jax", "native;algorithm=direct;backend=ipc"]
    cmd = [sys.executable, "-m", "ddlb_amd", "--primitive", primitive, "-m", "2048", "-n", "512",
           "-k", "1024", "--dtype", "bfloat16", "--num-iterations", "3", "--num-warmups", "1",
           "--output-csv", str(out)]
    for spec in impls:
        cmd += ["--impl", spec]
    env = _env()
    env["DDLB_MASTER_PORT"] = str(free_port())
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    files = list(tmp_path.glob("res_*.csv"))
    assert len(files) == 1, r.stdout[-2000:]
    with open(files[0], newline="") as f:
        reader = csv.DictReader(f)
        header = reader.fieldnames
        rows = list(reader)
    assert header[:len(CSV_COLUMNS)] == CSV_COLUMNS
    n_expected = 3 + 1 + 1 + 1 + 1 + 1 + (2 if primitive == "tp_columnwise" else 0)
    assert len(rows) == n_expected, [row["implementation"] for row in rows]
    bad = [(row["implementation"], row.get("error", "")) for row in rows
           if row["valid"] != "True"]
    assert not bad, bad
    for row in rows:
        assert float(row["mean_time (ms)"]) > 0 and float(row["Throughput (TFLOPS)"]) > 0
