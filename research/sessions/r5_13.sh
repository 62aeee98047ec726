# round 5 / 13: kernel stats of the K-split forms (why f32 partials cost 2x)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ks -- python3 -u scripts/ab_ksplit_forms.py --shapes 8192x1024x8192 --only 'ks2\[pt4\]/reduce' --rounds 2 > $O/ks_prof.txt 2>&1 || { echo "prof failed"; tail -30 $O/ks_prof.txt; exit 1; }
grep -v "^  check.* ok$" $O/ks_prof.txt | tail -8
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -12
