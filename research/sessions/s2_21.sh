set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_21_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2_21_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag_blas_tune.py > gpurun_out/s2_21_tune.log 2>&1 || { tail gpurun_out/s2_21_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s2_21_tune.log
