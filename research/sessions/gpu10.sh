set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/g10_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g10_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python scripts/bench_gemm.py --rounds 3 --iters 10 --tiles i256,pi256,i256w4,128x128 --json gpurun_out/g10_gemm_bf16.json > gpurun_out/g10_gemm_bf16.log 2>&1 || exit 4
