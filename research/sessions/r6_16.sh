# round 6 / 16: park + hold inside K-tile 0 only (4 held pairs stored after the load phases' DMA, the 4 parked ones after the MFMA phases: 8 stores per wave in the next tile's first K-tile, no run-time flag): lab A/B ref (committed park) vs base
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_16
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 300 python -u $L --variants ref,base --rounds 11 --shapes 65536x1024x1024,65536x1024x512,65536x1024x2048,8192x8192x8192 > $O/ab_hold0_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_hold0_bf16.txt; exit 1; }
cat $O/ab_hold0_bf16.txt
timeout -k 10 200 python -u $L --variants ref,base --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x512,65536x1024x2048 > $O/ab_hold0_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_hold0_mx.txt; exit 1; }
cat $O/ab_hold0_mx.txt
