# round 6 / 21: lgkm_g0 on the park kernel (lgkm0) and load phases at priority 2 (prioload) against the product kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_21
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
V=base,lgkm0,prioload
timeout -k 10 400 python -u $L --variants $V --rounds 9 --shapes 65536x1024x1024,65536x1024x4096,8192x8192x8192 > $O/ab_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_bf16.txt; exit 1; }
cat $O/ab_bf16.txt
timeout -k 10 300 python -u $L --variants $V --dtype mx --rounds 9 --shapes 65536x1024x1024,65536x1024x512,65536x1024x4096 > $O/ab_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_mx.txt; exit 1; }
cat $O/ab_mx.txt
