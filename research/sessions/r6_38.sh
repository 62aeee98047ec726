# round 6 / 38: the steady loop unrolled by two (unroll2) against the product kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_38
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,unroll2 --rounds 13 --shapes 65536x1024x1024,8192x8192x8192,65536x1024x4096 > $O/ab_unroll2_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_unroll2_bf16.txt; exit 1; }
grep -v "^/opt" $O/ab_unroll2_bf16.txt
timeout -k 10 300 python -u $L --variants base,unroll2 --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_unroll2_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_unroll2_mx.txt; exit 1; }
grep -v "^/opt" $O/ab_unroll2_mx.txt
