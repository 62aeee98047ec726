# round 6 / 28: the steady K-loop without the tile-crossing test (nocross) against the product kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_28
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,nocross --rounds 11 --shapes 65536x1024x1024,65536x1024x4096,8192x8192x8192,65536x1024x512 > $O/ab_nocross_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_nocross_bf16.txt; exit 1; }
cat $O/ab_nocross_bf16.txt
timeout -k 10 300 python -u $L --variants base,nocross --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_nocross_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_nocross_mx.txt; exit 1; }
cat $O/ab_nocross_mx.txt
