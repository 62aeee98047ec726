# After the raster default G=4: bf16 long-K / partial shapes and MX-fp8 vs hipBLASLt, numerics checked
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_10
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_gemm.py --check --tiles auto --shapes 0,2,4,5,6 --rounds 3 > $O/gemm_bf16.log 2>&1 || { tail $O/gemm_bf16.log; exit 1; }
grep -a "check\|native\|hipblaslt\|^[0-9]" $O/gemm_bf16.log
timeout -k 10 300 python -u scripts/bench_gemm.py --check --dtype float8_e4m3fn --tiles auto --modes mx --shapes 0,6 --rounds 3 > $O/gemm_mx.log 2>&1 || { tail $O/gemm_mx.log; exit 1; }
grep -a "check\|native\|hipblaslt\|^[0-9]" $O/gemm_mx.log
