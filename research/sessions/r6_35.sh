# round 6 / 35: the tile end's packing and stores of C rows mq = 0 interleaved with the last K-tile's
# remaining MFMAs (ilv) against the product kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_35
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,ilv --rounds 13 --shapes 65536x1024x1024,65536x1024x512,8192x8192x8192 > $O/ab_ilv_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_ilv_bf16.txt; exit 1; }
cat $O/ab_ilv_bf16.txt | grep -v "^/opt"
timeout -k 10 300 python -u $L --variants base,ilv --dtype mx --rounds 13 --shapes 65536x1024x1024,65536x1024x512 > $O/ab_ilv_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_ilv_mx.txt; exit 1; }
cat $O/ab_ilv_mx.txt | grep -v "^/opt"
