# round 6 / 33: branch-free steady K-tiles (waitall: both groups wait at all four vmcnt sites) for the MX
# kernel, which cannot take the per-group split (spills); bf16 beside it for information
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_33
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 300 python -u $L --variants base,waitall --dtype mx --rounds 13 --shapes 65536x1024x1024,65536x1024x4096,16384x8192x8192 > $O/ab_waitall_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_waitall_mx.txt; exit 1; }
cat $O/ab_waitall_mx.txt | grep -v "^/opt"
timeout -k 10 300 python -u $L --variants base,waitall --rounds 9 --shapes 65536x1024x1024,8192x8192x8192 > $O/ab_waitall_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_waitall_bf16.txt; exit 1; }
cat $O/ab_waitall_bf16.txt | grep -v "^/opt"
