"""Opt-in PMC collection of the runner (ddlb_amd/utils/pmc.py): counter-set validation (an
over-full rocprofv3 pass hangs, so it must be refused before launch), the launcher prefix, the
per-kernel summary of a rocpd database, and the standalone worker a profiler wraps."""

import json
import os
import sqlite3
import subprocess
import sys

import pytest

from ddlb_amd.utils import pmc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_and_default_set_fit_one_pass():
    assert pmc.parse("SQ_WAVES, GRBM_GUI_ACTIVE") == ["SQ_WAVES", "GRBM_GUI_ACTIVE"]
    assert pmc.parse(None) == [] and pmc.parse("") == []
    assert pmc.parse("default") == list(pmc.DEFAULT_SET)
    assert pmc.check_limits(pmc.DEFAULT_SET) == {"SQ": 8, "GRBM": 1}


def test_over_full_pass_is_refused():
    nine = [f"SQ_C{i}" for i in range(9)]
    with pytest.raises(ValueError, match="SQ: 9 > 8"):
        pmc.check_limits(nine)
    with pytest.raises(ValueError, match="TCC: 5 > 4"):
        pmc.check_limits(["FETCH_SIZE", "WRITE_SIZE"])
    assert pmc.check_limits(["FETCH_SIZE", "TCC_HIT_sum"]) == {"TCC": 4}
    # _sum/_avr of one counter occupy one slot
    assert pmc.check_limits(["TCC_HIT_sum", "TCC_HIT_avr", "TCC_MISS_sum"]) == {"TCC": 2}
    with pytest.raises(ValueError, match="unknown block"):
        pmc.check_limits(["FOO_BAR"])


def test_rocprof_prefix_runs_the_program_directly():
    cmd = pmc.rocprof_cmd(["SQ_WAVES"], "/tmp/x")
    assert cmd[1:3] == ["--pmc", "SQ_WAVES"] and "--selected-regions" in cmd
    assert cmd[-1] == "--"  # the program follows directly (no env / shell hop)
    assert not any(flag in cmd for flag in ("-s", "--sys-trace", "-r", "--runtime-trace"))


def test_summarize_rocpd(tmp_path):
    db = tmp_path / "a" / "pmc_results.db"
    db.parent.mkdir()
    con = sqlite3.connect(db)
    con.execute("create table counters_collection (kernel_name text, counter_name text, "
                "value real)")
    rows = [("void ddlb::(anonymous namespace)::gemm_tn_pt4_kernel<ddlb::MmaBF16, 2>(ddlb::G)",
             "SQ_WAVES", 2048.0)] * 2 + [("Cijk_Alik_Bljk_MT256x256x64_SK3", "SQ_WAVES", 1024.0)]
    con.executemany("insert into counters_collection values (?, ?, ?)", rows)
    con.commit()
    con.close()
    out = pmc.summarize(str(tmp_path))
    assert out["gemm_tn_pt4_kernel<ddlb::MmaBF16, 2>"]["SQ_WAVES"] == 2048.0
    assert out["hipBLASLt 256x256x64"]["SQ_WAVES"] == 1024.0


def test_runner_rejects_bad_pmc_before_any_child():
    from ddlb_amd.benchmark import PrimitiveBenchmarkRunner

    with pytest.raises(ValueError):
        PrimitiveBenchmarkRunner("tp_columnwise", 64, 64, 64, ["compute_only_0"],
                                 pmc=",".join(f"SQ_C{i}" for i in range(9)))


def test_standalone_worker_cpu(tmp_path):
    """The child a profiler launcher wraps: ``python -m ddlb_amd.benchmark --worker``."""
    from conftest import free_port

    kwargs = dict(primitive="tp_columnwise", impl_id="compute_only_0", m=64, n=32, k=16,
                  dtype="float32", num_warmups=1, num_iterations=2,
                  impl_opts={"implementation": "compute_only", "size": "unsharded"},
                  validate=True)
    jin, jout = tmp_path / "in.json", tmp_path / "out.json"
    jin.write_text(json.dumps(kwargs))
    env = dict(os.environ, DDLB_DEVICE="cpu",
               DDLB_CHILD_INIT_METHOD=f"tcp://127.0.0.1:{free_port()}")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "ddlb_amd.benchmark", "--worker", str(jin),
                        str(jout)], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    row = json.loads(jout.read_text())
    assert row["valid"] is True and row["mean_time (ms)"] > 0


def test_summarize_top(tmp_path):
    db = tmp_path / "pmc_results.db"
    con = sqlite3.connect(db)
    con.execute("create table counters_collection (kernel_name text, counter_name text, "
                "value real)")
    con.executemany("insert into counters_collection values (?, ?, ?)",
                    [(f"k{i}", "GRBM_GUI_ACTIVE", float(i)) for i in range(12)])
    con.commit()
    con.close()
    assert set(pmc.summarize(str(tmp_path), top=3)) == {"k11", "k10", "k9"}
