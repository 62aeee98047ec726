# product pt4 with the DEFER (balanced phases) schedule for ungated write-through kernels:
# GEMM numerics suite, GEMM vs hipBLASLt (bf16 + MX), bench N=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_32
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1; rc=$?; tail -3 $O/gemm_tests.log; grep -a "FAILED\|Timeout" $O/gemm_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm.py --check --tiles auto --shapes 0,2,4,5,6 --rounds 3 > $O/gemm_bf16.log 2>&1 || { tail $O/gemm_bf16.log; exit 1; }
grep -a "check\|native\|hipblaslt\|^[0-9]" $O/gemm_bf16.log
timeout -k 10 300 python -u scripts/bench_gemm.py --check --dtype float8_e4m3fn --tiles auto --modes mx --shapes 0,6 --rounds 3 > $O/gemm_mx.log 2>&1 || { tail $O/gemm_mx.log; exit 1; }
grep -a "check\|native\|hipblaslt\|^[0-9]" $O/gemm_mx.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench" $O/bench.log | cut -c1-200; grep metric $O/bench.log | cut -c1-400
