# round 6 / 13: the one-wave-per-SIMD geometry again (q4: 4 waves of 128x128, AGPR accumulators, research/lab/gemm_lab.hip) against today's product pt4, with its timing ablations: how far is the LDS-read saving from paying?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_13
mkdir -p $O
export TMPDIR=/tmp
for s in "8192 8192 8192" "65536 1024 1024" "65536 1024 4096"; do
  LAB_ONLY="q4 bufdma,q4s1 bufdma,q4 noDMA,q4 noBAR,q4 noMFMA,q4 noDMA noBAR,pt4v15" timeout -k 10 120 research/lab/bin/gemm_lab $s >> $O/q4.txt 2>&1 || { echo "gemm_lab failed"; tail -20 $O/q4.txt; exit 1; }
done
cat $O/q4.txt
timeout -k 10 200 python -u research/lab/pt4_ablate.py --variants base --rounds 5 --shapes 8192x8192x8192,65536x1024x1024,65536x1024x4096 > $O/pt4.txt 2>&1 || { echo "pt4 failed"; tail -20 $O/pt4.txt; exit 1; }
cat $O/pt4.txt
