# round 4 / 3: budget after the uncached local flags, with per-op timelines of the RCCL-fed fused
# plans and the top candidates; rocprofv3 kernel stats of the config-#4 budget
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_3
mkdir -p $O
export TMPDIR=/tmp
TL="coll_pipeline/rccl/s8/fused,coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8/fused/r48,default/rccl,coll_pipeline/rccl/s4,p2p_pipeline/rccl/fused"
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --timeline "$TL" --out $O/col8_tl.json > $O/col8_tl.txt 2>&1 || { echo "col8 failed"; tail -20 $O/col8_tl.txt; exit 1; }
cat $O/col8_tl.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o budget -- python -u scripts/plan_budget.py --world 8 --iters 10 --candidates "coll_pipeline/rccl/s8/fused,coll_pipeline/rccl/s8,direct/ipc,coll_pipeline/ipc/agk32/s4/graph" > $O/prof.txt 2>&1 || { echo "prof failed"; tail -20 $O/prof.txt; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
