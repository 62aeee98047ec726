# round 6 / 18: load-phase order (the 4 LDS-DMA pieces before the 12 fragment reads: dmafirst; between
# the B and A reads: dmamid) and no MFMA-phase priority (noprio) against the product kernel, one process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_18
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
V=base,dmafirst,dmamid,noprio
timeout -k 10 400 python -u $L --variants $V --rounds 9 --shapes 65536x1024x1024,65536x1024x4096,8192x8192x8192 > $O/ab_order_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_order_bf16.txt; exit 1; }
cat $O/ab_order_bf16.txt
timeout -k 10 300 python -u $L --variants $V --dtype mx --rounds 9 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_order_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_order_mx.txt; exit 1; }
cat $O/ab_order_mx.txt
