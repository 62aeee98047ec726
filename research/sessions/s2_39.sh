# Rehearsal after the raster / dispatch / nt-store changes: 8 ranks sharing the GPU (one HW queue
# each), the IPC candidates incl. the kernel-signal hedges, validated final run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="direct/ipc,p2p_pipeline/ipc/memcpy,coll_pipeline/ipc/memcpy/s4,default/ipc/kernel,default/ipc/kernel/blas,p2p_pipeline/ipc/push,coll_pipeline/ipc/push/s4,p2p_pipeline/ipc/memcpy/ksig,default/ipc/kernel/ksig"
GPU_MAX_HW_QUEUES=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 8 --steps 5 --warmup 2 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_39_b8.log 2>&1; rc=$?
echo "n=8 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_39_b8.log | cut -c1-150; grep -ao '"valid": [a-z]*\|"algorithm": "[^"]*"' gpurun_out/s2_39_b8.log; exit $rc
