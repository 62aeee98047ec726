set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_20_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2_20_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dtype float8_e4m3fn > gpurun_out/s2_20_fp8.log 2>&1 || { tail gpurun_out/s2_20_fp8.log; exit 1; }
grep -ao '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"algorithm": "[^"]*"\|"autotune_ms.*' gpurun_out/s2_20_fp8.log | tr '\n' ' '; echo
timeout -k 10 300 python scripts/bench_gemm.py --help > /dev/null 2>&1; true
