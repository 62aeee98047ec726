# round 5 / 17: whole GPU suite after the f32 store regrouping + K-split changes; smoke; bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_17
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
timeout -k 10 400 python bench.py -m 8192 -n 1024 -k 8192 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench c2 failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-300 $O/bench_c2_bf16.json
