# round 4 / 32: reserve_cus of the RCCL-fed fused GEMM (CUs left to the collectives): 16 / 32 /
# 48 / 64 in the emulated d = 8 budget, fast (32-block) and link-like (6-block) stand-ins
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_32
mkdir -p $O
TL="coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8/fused,p2p_pipeline/rccl/fused"
V="reserve_cus=16;reserve_cus=48;reserve_cus=64"
for b in 32 6; do
  timeout -k 10 300 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --variants "$V" --rccl-blocks $b --iters 30 > $O/b$b.txt 2>&1 || { echo "budget failed"; tail -20 $O/b$b.txt; exit 1; }
  echo "== blocks $b"; grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp\|^EMULATED" $O/b$b.txt
done
