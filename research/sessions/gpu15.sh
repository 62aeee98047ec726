set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/g15_tests.log 2>&1; rc=$?; tail -5 gpurun_out/g15_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_gemm.py --tiles i256,pi256,r256,128x128 --json gpurun_out/g15_gemm_bf16.json > gpurun_out/g15_gemm_bf16.log 2>&1; echo "gemm rc=$?"; grep -v amdgpu.ids gpurun_out/g15_gemm_bf16.log
timeout -k 10 300 python scripts/bench_gemm.py --dtype float8_e4m3fn --tiles i256,r256 --shapes 0,2,6 > gpurun_out/g15_gemm_fp8.log 2>&1; echo "fp8 rc=$?"; grep -v amdgpu.ids gpurun_out/g15_gemm_fp8.log
