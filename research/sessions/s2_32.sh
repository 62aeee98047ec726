# Grouped tile raster for t8/pt8/t4/pt4: numerics of the four kernels, then timings vs hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "t8 or pt4 or t4" > gpurun_out/s2_32_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s2_32_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/diag_blas_tune.py > gpurun_out/s2_32_tune.log 2>&1 || { tail gpurun_out/s2_32_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s2_32_tune.log
