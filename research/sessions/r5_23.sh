# round 5 / 23: TIMING-ONLY ablation (wrong results by design): pt4 with two wave-group
# hand-offs per K-tile instead of four (DDLB_PT4_ABLATE_MERGE=1) -- what the hand-offs cost
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_23
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_ABLATE_MERGE --values unset,1 --shapes 0,2,5,6 --rounds 3 > $O/ab_ablate_merge.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab_ablate_merge.txt; exit 1; }
grep -A4 "median" $O/ab_ablate_merge.txt
