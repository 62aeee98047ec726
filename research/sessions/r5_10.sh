# round 5 / 10: config #2 shape (8192x1024x8192, 128 256x256 tiles): the auto K-split (pt4,
# S=2, in-launch reduce) against unsplit smaller tiles that fill the chip in one pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 3 --check --rounds 5 --tiles auto,pt4,256x128,128x256,i128,256x128w4,128x128 > $O/gemm_c2_tiles_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/gemm_c2_tiles_bf16.txt; exit 1; }
cat $O/gemm_c2_tiles_bf16.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 3 --check --rounds 5 --dtype float8_e4m3fn --modes mx --tiles auto,pt4,256x128,128x256,128x128 > $O/gemm_c2_tiles_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/gemm_c2_tiles_mx.txt; exit 1; }
cat $O/gemm_c2_tiles_mx.txt
