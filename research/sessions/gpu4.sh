set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/g4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g4_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_gemm.py --rounds 3 --iters 10 --json gpurun_out/g4_gemm_bf16.json > gpurun_out/g4_gemm_bf16.log 2>&1 || exit 4
timeout -k 10 200 python scripts/bench_gemm.py --dtype float8_e4m3fn --rounds 3 --iters 10 --tiles pp256,256x256 --modes auto,mx --shapes 0,2,6 > gpurun_out/g4_gemm_fp8.log 2>&1 || exit 5
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/g4_bench.log 2>&1; tail -1 gpurun_out/g4_bench.log
