# round 6 / 24: what the A stream from HBM costs (al2: A from two L2-resident panels, al2ns: and no C
# stores, nostore) and K-rotation across the four CUs that share an A panel (krot), against the product
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_24
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,krot,nostore,al2,al2ns --rounds 9 --shapes 65536x1024x1024,16384x1024x1024,65536x1024x4096 > $O/ab_a_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_a_bf16.txt; exit 1; }
cat $O/ab_a_bf16.txt
timeout -k 10 300 python -u $L --variants base,krot,nostore,al2,al2ns --dtype mx --rounds 9 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_a_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_a_mx.txt; exit 1; }
cat $O/ab_a_mx.txt
