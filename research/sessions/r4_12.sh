# round 4 / 12: RCCL-fed fused plans, A/B of signal placement (comm stream vs a third stream) and
# GEMM-first enqueue, with fast (32-block) and link-like slow (6-block) emulated collectives
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_12
mkdir -p $O
export TMPDIR=/tmp
TL="coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8/fused,p2p_pipeline/rccl/fused,coll_pipeline/rccl/s4"
V="sig_side=0;gemm_first=0;sig_side=0,gemm_first=0"
for b in 32 6; do
  timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --variants "$V" --rccl-blocks $b --iters 30 --out $O/ab_b$b.json > $O/ab_b$b.txt 2>&1 || { echo "budget b$b failed"; tail -20 $O/ab_b$b.txt; exit 1; }
  grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp" $O/ab_b$b.txt
done
