# round 5 / 36: the final in-tree .so (rebuilt after comment / whitespace edits): GEMM + K-split
# + knob tests, smoke, bench N=1 bf16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_36
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_native_gpu.py tests/test_reduce_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
