# round 5 / 7: K-split tests (split + reduce default, in-launch reduction opt-in, one quadrant of
# loads at a time), config #2 bench (default form), flagship bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py tests/test_gemm_gpu.py -k "ksplit or split_k or gated or queue_pools" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 300 python bench.py -m 8192 -n 1024 -k 8192 --steps 50 --warmup 10 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-300 $O/bench_c2_bf16.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
