# Session-end verification: GPU suite, smoke, bench N=1 (bf16 flagship, fp8 config #5 dtype,
# tp_rowwise config #3 shape), rocprofv3 kernel stats of the flagship bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_16
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" $O/gpu_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bf16.log 2>&1 || { echo bench failed; tail -20 $O/bench_bf16.log; exit 1; }
grep -a "\[bench\]" $O/bench_bf16.log; grep metric $O/bench_bf16.log | cut -c1-260
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.log 2>&1 || { echo bench fp8 failed; tail -20 $O/bench_fp8.log; exit 1; }
grep -a "\[bench\]" $O/bench_fp8.log; grep metric $O/bench_fp8.log | cut -c1-260
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > $O/bench_row.log 2>&1 || { echo bench row failed; tail -20 $O/bench_row.log; exit 1; }
grep -a "\[bench\]" $O/bench_row.log; grep metric $O/bench_row.log | cut -c1-260
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python bench.py --steps 50 --algorithm "gemm (world=1)/hip" > $O/prof.log 2>&1; echo "prof rc=$?"
find $O/prof -name "*kernel_stats.csv" | head -2
