# round 6 / 39: end-of-round validation of the final tree: whole GPU suite, smoke, bench.py N=1 with the
# driver's arguments (bf16, fp8) and with no arguments (the driver's default form)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_39
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; grep -v "^  File\|^    " $O/gpu_tests.txt | tail -40; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
grep "tune\|final" $O/bench_bf16.err | cut -c1-120
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-300 $O/bench_fp8.json
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench default failed"; tail -20 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
