# round 6 / 42: BASELINE config #2 shape at N=1 on the final tree (tp_columnwise m=8192 n=1024 k=8192; bf16, fp8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_42
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 -m 8192 -n 1024 -k 8192 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-260 $O/bench_c2_bf16.json
grep "tune\|final" $O/bench_c2_bf16.err | cut -c1-120
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 -m 8192 -n 1024 -k 8192 --dtype float8_e4m3fn > $O/bench_c2_fp8.json 2> $O/bench_c2_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_c2_fp8.err; exit 1; }
cut -c1-260 $O/bench_c2_fp8.json
grep "tune\|final" $O/bench_c2_fp8.err | cut -c1-120
