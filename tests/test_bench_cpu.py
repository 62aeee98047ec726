"""bench.py orchestration on the CPU: parent/child process model, gloo coordination, MAX over
ranks, the one-line JSON contract (GPU-free path: the pytorch candidate on gloo)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "3", "--warmup", "1", "-m", "256", "-n", "64", "-k", "64",
        "--algorithm", "pytorch(rccl+hipblaslt)", "--dtype", "float32"]


def _json_line(out: str):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    env = dict(os.environ, DDLB_DEVICE="cpu")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "DDLB_CHILD_INIT_METHOD"):
        env.pop(k, None)
    return env


def test_bench_world1_cpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in d
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["valid"] is True
    assert d["value"] > 0 and d["scaling"] == "weak"


def test_bench_world2_cpu():
    from conftest import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=_env())
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["valid"] is True
    assert abs(d["value"] - 2 * d["per_gpu_tflops"]) < 1e-2
