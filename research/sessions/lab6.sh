set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 scripts/lab/bin/gemm_lab 65536 1024 1024 > gpurun_out/lab6_a.log 2>&1; rc=$?; cat gpurun_out/lab6_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python scripts/diag_blas.py > gpurun_out/lab6_blas.log 2>&1; grep -v amdgpu.ids gpurun_out/lab6_blas.log
