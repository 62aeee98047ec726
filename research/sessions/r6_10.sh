# round 6 / 10: PARK, second session (kill rule): lab A/B ref (committed) vs base (park) with more rounds, plus a one-tile-per-workgroup shape (the final drain) and K = 2048; then bench.py N=1 bf16 and fp8 on the park tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_10
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 300 python -u $L --variants ref,base --rounds 11 --shapes 65536x1024x1024,16384x1024x1024,65536x1024x2048,65536x1024x512 > $O/ab_park_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_park_bf16.txt; exit 1; }
cat $O/ab_park_bf16.txt
timeout -k 10 200 python -u $L --variants ref,base --dtype mx --rounds 11 --shapes 65536x1024x1024,16384x1024x1024,65536x1024x2048 > $O/ab_park_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_park_mx.txt; exit 1; }
cat $O/ab_park_mx.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-300 $O/bench_fp8.json
