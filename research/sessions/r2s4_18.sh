# pt4 write-through (sc1 | nt) C stores in the product: A/B vs plain nt stores, numerics, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_18
mkdir -p $O
F="amdgpu.ids\|socket.cpp"
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gemm_tests.log 2>&1; rc=$?; tail -2 $O/gemm_tests.log; [ $rc -eq 0 ] || { grep -a "FAIL\|Error" $O/gemm_tests.log | tail -20; exit $rc; }
for v in wt nt wt nt; do
  if [ $v = nt ]; then export DDLB_PT4_NT_STORES=1; else unset DDLB_PT4_NT_STORES; fi
  timeout -k 10 300 python scripts/bench_gemm.py --rounds 3 --iters 20 --tiles auto --modes auto,blas --shapes 0,1,2,3 > $O/gemm_$v.log 2>&1; rc=$?; echo "== C stores: $v"; grep -v "$F" $O/gemm_$v.log | grep "native\|bfloat16\|hipblaslt" | head -16; [ $rc -eq 0 ] || exit $rc
done
unset DDLB_PT4_NT_STORES
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench\]" $O/bench.log; grep metric $O/bench.log | cut -c1-250
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.log 2>&1 || { echo bench fp8 failed; tail -20 $O/bench_fp8.log; exit 1; }
grep -a "\[bench\]" $O/bench_fp8.log; grep metric $O/bench_fp8.log | cut -c1-250
