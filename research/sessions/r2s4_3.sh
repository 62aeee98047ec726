# CU copy kernel 4 vs 8 loads in flight per lane; GPU suite; 2-rank shared-GPU rehearsal of the
# agk candidates with the write-through copy role (ag_mode 6 default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_3
mkdir -p $O
F="amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl"
DDLB_COPY_U=4 timeout -k 10 200 python scripts/bench_reduce.py --copy > $O/copy_u4.log 2>&1 || { tail $O/copy_u4.log; exit 1; }
timeout -k 10 200 python scripts/bench_reduce.py --copy > $O/copy_u8.log 2>&1 || { tail $O/copy_u8.log; exit 1; }
echo "U=4"; grep -v "$F" $O/copy_u4.log; echo "U=8"; grep -v "$F" $O/copy_u8.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk64/s8/graph,coll_pipeline/ipc/agk32/s4/graph,coll_pipeline/ipc/agk32/s8,coll_pipeline/ipc/memcpy/s8/graph,coll_pipeline/ipc/kernel/s8/graph"
start=$(date +%s)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
echo "2 ranks rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" $O/bench2.log | cut -c1-220
exit $rc
