# round 6 / 15: C store cache policy again with the park (the tile-end burst is 12 stores per wave now): bf16 and MX flagship, K = 512
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_15
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 200 python -u $L --variants base,aux3,aux17,aux19 --rounds 9 --shapes 65536x1024x1024,65536x1024x512 > $O/ab_cpol_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_cpol_bf16.txt; exit 1; }
cat $O/ab_cpol_bf16.txt
timeout -k 10 200 python -u $L --variants base,aux3,aux18,aux19 --dtype mx --rounds 9 --shapes 65536x1024x1024,65536x1024x512 > $O/ab_cpol_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_cpol_mx.txt; exit 1; }
cat $O/ab_cpol_mx.txt
