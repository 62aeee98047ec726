# round 6 / 34: long K against the vendor in one process on the final kernel (stage_ab + SPLIT): bf16 65536x1024x8192, 16384x8192x8192, 8192^3, flagship; MX 65536x1024x8192, 16384x8192x8192, flagship vs _scaled_mm; bench.py tp_rowwise config #3 at N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_34
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 2,5,6,0 --tiles auto --rounds 9 --check --json $O/longk_bf16.json > $O/longk_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/longk_bf16.txt; exit 1; }
grep -v "^/opt" $O/longk_bf16.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --dtype float8_e4m3fn --modes mx --shapes 2,5,0 --tiles auto --rounds 9 --check --json $O/longk_mx.json > $O/longk_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/longk_mx.txt; exit 1; }
grep -v "^/opt" $O/longk_mx.txt
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > $O/bench_row3.json 2> $O/bench_row3.err || { echo "bench row failed"; tail -20 $O/bench_row3.err; exit 1; }
cut -c1-300 $O/bench_row3.json
grep "tune\|final" $O/bench_row3.err | cut -c1-160
