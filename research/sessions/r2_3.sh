# Round 2: multi-rank rehearsal of bench.py after the validated-autotune / uncached-flag changes.
# Ranks share the box's one GPU (gloo control plane; RCCL candidates fail fast by design there).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
start=$(date +%s)
GPU_MAX_HW_QUEUES=2 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --steps 10 --warmup 3 --candidate-timeout 60 > gpurun_out/r2/r2_3_bench4.log 2>&1; rc=$?
echo "4 ranks rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" gpurun_out/r2/r2_3_bench4.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
C="direct/ipc,p2p_pipeline/ipc/memcpy,coll_pipeline/ipc/memcpy/s4,default/ipc/kernel,p2p_pipeline/ipc/push,default/ipc/kernel/ksig"
start=$(date +%s)
GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 8 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/r2/r2_3_bench8.log 2>&1; rc=$?
echo "8 ranks rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" gpurun_out/r2/r2_3_bench8.log | cut -c1-300
exit $rc
