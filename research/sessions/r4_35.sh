# round 4 / 35: validation of the final tree (after the gated-reserve floor and the CU-filling rccl_fused preflight): GPU suite, smoke, bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_35
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-250 $O/bench_bf16.json
