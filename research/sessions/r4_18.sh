# round 4 / 18: gated pt4 grid shrink (fewest workgroups keeping the tile-round count) vs the full
# num_cus - reserve grid, emulated budget with fast (32-block) and link-like (6-block) collectives
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_18
mkdir -p $O
TL="coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8/fused,p2p_pipeline/rccl/fused,coll_pipeline/ipc/memcpy/s8/fused"
for b in 32 6; do
  for ns in 0 1; do
    if [ $ns = 1 ]; then export DDLB_PT4_NO_SHRINK=1; else unset DDLB_PT4_NO_SHRINK; fi
    timeout -k 10 300 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --rccl-blocks $b --iters 30 > $O/b${b}_noshrink$ns.txt 2>&1 || { echo "budget failed"; tail -20 $O/b${b}_noshrink$ns.txt; exit 1; }
    echo "== blocks $b no_shrink $ns"; grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp\|^EMULATED\|^candidate" $O/b${b}_noshrink$ns.txt
  done
done
