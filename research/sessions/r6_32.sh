# round 6 / 32: one M0 per unit slice (m0share: the second 1 KB DMA piece through the instruction offset)
# against the product kernel; exact only if that offset also offsets the LDS address (the check says)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_32
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,m0share --rounds 13 --shapes 65536x1024x1024,8192x8192x8192,65536x1024x512 > $O/ab_m0_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_m0_bf16.txt; exit 1; }
cat $O/ab_m0_bf16.txt | grep -v "^/opt"
timeout -k 10 300 python -u $L --variants base,m0share --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_m0_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_m0_mx.txt; exit 1; }
cat $O/ab_m0_mx.txt | grep -v "^/opt"
