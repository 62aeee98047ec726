# round 6 / 23: phase stamps (pstamps): which side of each barrier waits -- the load phase (reads +
# DMA issue, then its lgkmcnt / vmcnt waits) or the MFMA phase -- bf16 one tile per workgroup, the
# flagship and K = 4096; MX flagship
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_23
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 300 python -u $L --variants base,pstamps --rounds 3 --stamp-report --shapes 16384x1024x1024,65536x1024x1024,65536x1024x4096 > $O/pstamps_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/pstamps_bf16.txt; exit 1; }
cat $O/pstamps_bf16.txt
timeout -k 10 300 python -u $L --variants base,pstamps --dtype mx --rounds 3 --stamp-report --shapes 65536x1024x1024,65536x1024x4096 > $O/pstamps_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/pstamps_mx.txt; exit 1; }
cat $O/pstamps_mx.txt
