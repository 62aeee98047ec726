set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_17_tests.log 2>&1; rc=$?; tail -5 gpurun_out/s2_17_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/diag_blas_tune.py > gpurun_out/s2_17_tune.log 2>&1 || { tail gpurun_out/s2_17_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s2_17_tune.log
timeout -k 10 300 python bench.py > gpurun_out/s2_17_bench.log 2>&1 || { tail gpurun_out/s2_17_bench.log; exit 1; }
grep -a "^{" gpurun_out/s2_17_bench.log | cut -c1-200; grep -ao '"autotune_ms.*' gpurun_out/s2_17_bench.log
