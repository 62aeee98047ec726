# round 4 / 19: validation after the gated grid shrink revert: GPU suite, budget of the leading
# candidates, 2-rank shared-GPU rehearsal (IPC families)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_19
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
TL="coll_pipeline/rccl/s4/fused,coll_pipeline/ipc/agk32/s4/graph,direct/ipc,coll_pipeline/rccl/s8/fused,coll_pipeline/rccl/s4,default/rccl,p2p_pipeline/rccl/fused,coll_pipeline/ipc/memcpy/s4/graph"
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --out $O/col8.json > $O/col8.txt 2>&1 || { echo "budget failed"; tail -20 $O/col8.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp" $O/col8.txt
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s4/graph,direct/ipc,coll_pipeline/ipc/memcpy/s8/fused,default/ipc/kernel"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29737 bench.py --gpus 2 --steps 20 --warmup 5 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
