# Rehearsal of the N>1 bench with the pt4/t4 GEMMs: 2 ranks (default queues) and 8 ranks (one HW
# queue each) sharing the one GPU, every IPC candidate, validated final runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="direct/ipc,p2p_pipeline/ipc/memcpy,p2p_pipeline/ipc/memcpy/blas,coll_pipeline/ipc/memcpy/s4,default/ipc/kernel,default/ipc/kernel/blas,p2p_pipeline/ipc/push,p2p_pipeline/ipc/push/blas,default/ipc/push,coll_pipeline/ipc/push/s4,default/ipc/kernel/push"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_25_b2.log 2>&1; rc=$?
echo "n=2 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_25_b2.log | cut -c1-150; grep -ao '"valid": [a-z]*' gpurun_out/s2_25_b2.log; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 8 --steps 5 --warmup 2 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_25_b8.log 2>&1; rc=$?
echo "n=8 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_25_b8.log | cut -c1-150; grep -ao '"valid": [a-z]*' gpurun_out/s2_25_b8.log; exit $rc
