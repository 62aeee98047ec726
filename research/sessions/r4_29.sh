# round 4 / 29: K-split in the per-shard / full GEMMs of the long-K configs: emulated d = 8
# budget at k = 8192 (BASELINE 4b), 2 ranks sharing the GPU at the config #2 shape (validated)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_29
mkdir -p $O
export TMPDIR=/tmp
TL="p2p_pipeline/rccl,p2p_pipeline/rccl/fused,coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8,default/rccl,direct/ipc"
timeout -k 10 500 python -u scripts/plan_budget.py --world 8 -k 8192 --candidates "$TL" > $O/col8_k8192.txt 2>&1 || { echo "budget failed"; tail -20 $O/col8_k8192.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp" $O/col8_k8192.txt
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="p2p_pipeline/ipc/memcpy/graph,default/ipc/kernel,direct/ipc"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29761 bench.py --gpus 2 -m 8192 -n 1024 -k 8192 --steps 10 --warmup 3 --candidates "$C" > $O/bench2_c2.log 2>&1; rc=$?
grep -a "tune\|final" $O/bench2_c2.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
