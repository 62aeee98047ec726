# round 4 / 23: ops-level K-split: full GPU suite, GEMM table on the few-tile long-K shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_23
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 3,0,2 --tiles auto,pt4,t4 --rounds 5 --check > $O/bf16.txt 2>&1 || { echo "bf16 failed"; tail -20 $O/bf16.txt; exit 1; }
grep -v amdgpu.ids $O/bf16.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --dtype float8_e4m3fn --shapes 3,0 --tiles auto,t4 --modes mx --rounds 5 --check > $O/fp8.txt 2>&1 || { echo "fp8 failed"; tail -20 $O/fp8.txt; exit 1; }
grep -v amdgpu.ids $O/fp8.txt
