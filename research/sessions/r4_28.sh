# round 4 / 28: final validation of the round-4 tree: GPU suite, smoke, bench N=1 bf16 / fp8 /
# config #2 shape / rowwise config #3 shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_28
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-250 $O/bench_bf16.json
timeout -k 10 400 python bench.py --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-250 $O/bench_fp8.json
timeout -k 10 400 python bench.py --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > $O/bench_row.json 2> $O/bench_row.err || { echo "bench row failed"; tail -20 $O/bench_row.err; exit 1; }
cut -c1-250 $O/bench_row.json
