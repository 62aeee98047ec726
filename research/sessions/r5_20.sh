# round 5 / 20: stress of the in-kernel all-gather publication forms (100 launches each, NaN
# before every launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/diag_agk_stress.py --runs 100 --modes 0,1,6,14,30 --graph 1 > $O/agk_stress_graph.txt 2>&1 || { echo "stress failed"; tail -20 $O/agk_stress_graph.txt; exit 1; }
grep "^{" $O/agk_stress_graph.txt
timeout -k 10 400 python -u scripts/diag_agk_stress.py --runs 100 --modes 0,6 --graph 0 > $O/agk_stress_eager.txt 2>&1 || { echo "stress failed"; tail -20 $O/agk_stress_eager.txt; exit 1; }
grep "^{" $O/agk_stress_eager.txt
