set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 scripts/lab/bin/gemm_lab 65536 1024 1024 > gpurun_out/lab1_a.log 2>&1; rc=$?; cat gpurun_out/lab1_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 scripts/lab/bin/gemm_lab 8192 8192 8192 > gpurun_out/lab1_b.log 2>&1; rc=$?; cat gpurun_out/lab1_b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm.py --tiles i256,pi256 --shapes 0,6 > gpurun_out/lab1_ref.log 2>&1; grep -v amdgpu.ids gpurun_out/lab1_ref.log
