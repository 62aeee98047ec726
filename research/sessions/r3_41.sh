# bench.py N=1 for BASELINE config #5's dtype (fp8 e4m3, MX kernel) and the tp_rowwise config #3 shape, final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_41
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.log 2>&1 || { tail -20 $O/bench_fp8.log; exit 1; }
grep -a "\[bench" $O/bench_fp8.log | cut -c1-160; grep -a metric $O/bench_fp8.log | cut -c1-700
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > $O/bench_row.log 2>&1 || { tail -20 $O/bench_row.log; exit 1; }
grep -a "\[bench" $O/bench_row.log | cut -c1-160; grep -a metric $O/bench_row.log | cut -c1-700
