# 8 ranks on one GPU with ONE hardware queue per process (more queues oversubscribe the HWS with
# 8 processes and the cross-process stream waits of the memcpy protocol stall: scripts/gpu/s2_8.sh).
# Checks every IPC candidate's d=8 protocol at the flagship shape; timings are meaningless.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo GPU_MAX_HW_QUEUES=1
C="direct/ipc,p2p_pipeline/ipc/memcpy,p2p_pipeline/ipc/memcpy/blas,p2p_pipeline/ipc/memcpy/fused,coll_pipeline/ipc/memcpy/s4,coll_pipeline/ipc/memcpy/s4/blas,default/ipc/kernel"
start=$(date +%s)
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 8 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_9_bench8.log 2>&1; rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" gpurun_out/s2_9_bench8.log | cut -c1-300
