# Non-temporal C stores in the product kernels: GEMM numerics, timings vs hipBLASLt, N=1 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_38_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s2_38_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/diag_blas_tune.py > gpurun_out/s2_38_tune.log 2>&1 || { tail gpurun_out/s2_38_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s2_38_tune.log
timeout -k 10 300 python bench.py > gpurun_out/s2_38_bench.log 2>&1 || { tail gpurun_out/s2_38_bench.log; exit 1; }
grep -a "\[bench\]" gpurun_out/s2_38_bench.log; grep -ao '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gemm": "[^"]*"' gpurun_out/s2_38_bench.log | tr '\n' ' '; echo
