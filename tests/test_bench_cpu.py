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


def _prewarm_worker(rank, world, port, q):
    import time

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), DDLB_DEVICE="cpu",
                      DDLB_CHILD_INIT_METHOD=f"tcp://127.0.0.1:{port}")
    sys.path.insert(0, ROOT)
    import bench
    from ddlb_amd.communicator import Communicator

    class SlowOnRank1:  # rank 1's run() is 4x slower: a wall-clock prewarm would diverge
        def run(self):
            time.sleep(0.004 if rank == 1 else 0.001)

    comm = Communicator()
    comm.ensure_process_group()
    q.put((rank, bench.prewarm_runs(SlowOnRank1(), comm, prewarm_ms=40.0)))
    comm.destroy()


def test_prewarm_runs_agree_across_ranks():
    """Every rank must issue the same number of run() calls (each holds collectives / epoch-
    matched signals): the pre-warm count is MAX-reduced, not taken from each rank's clock."""
    import multiprocessing as mp

    from conftest import free_port

    ctx = mp.get_context("spawn")
    q, port = ctx.Queue(), free_port()
    procs = [ctx.Process(target=_prewarm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert got[0] == got[1] and got[0] >= 30, got


def test_bench_rowwise_world2_cpu():
    """--primitive tp_rowwise: GEMM + reduce-scatter; strong scaling, so the whole-job value is
    the reference harness number itself (ranks share one [m,k]x[k,n])."""
    from conftest import free_port

    args = ["--steps", "3", "--warmup", "1", "-m", "256", "-n", "64", "-k", "64", "--dtype",
            "float32", "--primitive", "tp_rowwise", "--algorithm", "row/pytorch(rccl+hipblaslt)"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=_env())
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["valid"] is True and d["scaling"] == "strong"
    assert d["metric"].startswith("tp_rowwise")
    assert abs(d["value"] - d["harness_tflops"]) < 1e-6
    assert abs(d["per_gpu_tflops"] - d["harness_tflops"] / 2) < 1e-6


def test_candidate_pools():
    sys.path.insert(0, ROOT)
    import bench

    col8 = bench.candidate_pool("tp_columnwise", "bfloat16", 8)
    assert any(c[0] == "direct/ipc" for c in col8) and all(c[0][:4] != "row/" for c in col8)
    row1 = bench.candidate_pool("tp_rowwise", "bfloat16", 1)
    assert [c[0] for c in row1] == ["row/gemm (world=1)/hip", "row/gemm (world=1)/blas"]
    fp8 = bench.candidate_pool("tp_columnwise", "float8_e4m3fn", 1)
    labels = [c[0] for c in fp8]
    assert "gemm (world=1)/hip/mx" in labels and not any("blas" in x for x in labels)
