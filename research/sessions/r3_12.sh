# pt4 deferred C stores (DDLB_PT4_DEFER=1/2): bit-identity tests, then an interleaved in-process A/B on the flagship / long-K / MX shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_12
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -v --timeout 120 --timeout-method thread -k "deferred or long_k_tight or persistent or fused_activation" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; grep -a "FAILED\|Timeout" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm.py --check --tiles auto --defer 0,1,2 --shapes 0,2,5,6 --rounds 5 > $O/bf16.log 2>&1 || { tail $O/bf16.log; exit 1; }
grep -a "check\|native\|hipblaslt\|^[0-9]" $O/bf16.log
timeout -k 10 200 python -u scripts/bench_gemm.py --check --dtype float8_e4m3fn --tiles auto --modes mx --defer 0,1,2 --shapes 0,6 --rounds 5 > $O/mx.log 2>&1 || { tail $O/mx.log; exit 1; }
grep -a "check\|native\|scaled\|^[0-9]" $O/mx.log
