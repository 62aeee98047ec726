# round 6 / 31: the tile loop split per wave group in the product (SPLIT), second session: lab A/B ref (HEAD) vs base
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_31
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants ref,base --rounds 13 --shapes 65536x1024x1024,8192x8192x8192,16384x8192x8192,65536x1024x512 > $O/ab_split_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_split_bf16.txt; exit 1; }
grep -v "check: max" $O/ab_split_bf16.txt
timeout -k 10 300 python -u $L --variants ref,base --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_split_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_split_mx.txt; exit 1; }
grep -v "check: max" $O/ab_split_mx.txt
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; grep -v "^  File\|^    " $O/gpu_tests.txt | tail -40; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
grep "tune\|final" $O/bench_bf16.err | cut -c1-120
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-300 $O/bench_fp8.json
