# round 5 / 2: in-launch K-split reduction (GemmArgs::ks_ws): GPU tests, config #2 shape through
# ops.gemm (auto = fused split) vs hipBLASLt and the old partial form (t4 slices + reduce),
# bench.py at the config #2 shape (bf16, MX-fp8), kernel-trace stats (one kernel, no reduce)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py tests/test_gemm_gpu.py -k "ksplit or split_k" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 3,0 --tiles auto,pt4 --rounds 5 --check > $O/gemm_c2.txt 2>&1 || { echo "bench_gemm failed"; tail -20 $O/gemm_c2.txt; exit 1; }
grep -E "x|ms" $O/gemm_c2.txt | head -20
timeout -k 10 300 python bench.py -m 8192 -n 1024 -k 8192 --steps 50 --warmup 10 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-300 $O/bench_c2_bf16.json
timeout -k 10 300 python bench.py -m 8192 -n 1024 -k 8192 --dtype float8_e4m3fn --steps 50 --warmup 10 > $O/bench_c2_fp8.json 2> $O/bench_c2_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_c2_fp8.err; exit 1; }
cut -c1-300 $O/bench_c2_fp8.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/scripts/bench_gemm.py --shapes 3 --tiles auto --rounds 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*stats*" | head
