# round 4 / 13: pt4 start-stagger A/B (half the CUs half a tile out of phase)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/ab_pt4_stagger.py --ns 0,2000,4000,7000,12000 --rounds 7 > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
