# round 4 / 20: K-split of few-tile long-K full GEMMs (BASELINE config #2 shape at N=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_20
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py -k "split_k or world1" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 400 python bench.py -m 8192 -n 1024 -k 8192 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2_bf16.json').read()); print(d['ms_per_step'], d['config']['algorithm'], d['autotune_ms'])"
timeout -k 10 400 python bench.py -m 8192 -n 1024 -k 8192 --dtype float8_e4m3fn > $O/bench_c2_fp8.json 2> $O/bench_c2_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_c2_fp8.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2_fp8.json').read()); print(d['ms_per_step'], d['config']['algorithm'], d['autotune_ms'])"
