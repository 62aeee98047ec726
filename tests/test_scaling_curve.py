"""scripts/scaling_curve.py: launch contract, JSON/CSV parsing and the efficiency table."""

import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location(
        "ddlb_scaling", os.path.join(ROOT, "scripts", "scaling_curve.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _line(n, ms, scaling="weak"):
    value = n * 137.4 / ms if scaling == "weak" else 137.4 / ms
    return json.dumps({"metric": "m", "value": value, "unit": "TFLOP/s", "n_gpus": n,
                       "steps": 5, "warmup": 1, "ms_per_step": ms, "scaling": scaling,
                       "dtype": "bf16", "config": {"model": "col", "algorithm": "a"}})


def test_bench_command_contract():
    m = _mod()
    one = m.bench_command(1, 5, 2, [], 1234)
    assert one[1].endswith("bench.py") and one[2:] == ["--gpus", "1", "--steps", "5", "--warmup", "2"]
    eight = m.bench_command(8, 5, 2, ["--dtype", "float8_e4m3fn"], 1234)
    assert eight[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in eight and "127.0.0.1" in eight and eight[-2:] == ["--dtype",
                                                                                    "float8_e4m3fn"]


def test_weak_and_strong_efficiency(tmp_path):
    m = _mod()
    f = tmp_path / "scale.jsonl"
    f.write_text("noise\n" + "\n".join([_line(1, 0.1), _line(2, 0.1), _line(8, 0.2)]) + "\n")
    rows = m.load([str(f)])
    table = m.render(rows)
    assert "| 1 | 0.1000 |" in table and "100.0 %" in table and "50.0 %" in table
    strong = [m._bench_row(json.loads(_line(n, ms, "strong"))) for n, ms in ((1, 0.8), (4, 0.25))]
    assert abs(m.efficiency(strong[1], strong[0]) - 0.8) < 1e-9


def test_csv_rows_and_best_per_key(tmp_path):
    m = _mod()
    f = tmp_path / "r.csv"
    hdr = "implementation,mean_time (ms),m,n,k,dtype,Throughput (TFLOPS),world_size,option,valid,error"
    f.write_text(hdr + "\n"
                 '"native (a)",0.5,8192,1024,8192,bfloat16,275.0,2,a,True,\n'
                 '"native (b)",0.4,8192,1024,8192,bfloat16,343.6,2,b,True,\n'
                 '"native (c)",0.1,8192,1024,8192,bfloat16,999.0,2,c,False,\n'
                 '"native (d)",,8192,1024,8192,bfloat16,,4,d,,boom\n')
    best = m.best_per_key(m.load([str(f)]))
    (label, by_n), = best.items()
    assert list(by_n) == [2] and by_n[2]["ms"] == 0.4
