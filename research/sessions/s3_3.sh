# Session 3: tp_rowwise (BASELINE config #3 shape, m=16384 n=8192 k=8192 bf16) with 2 ranks sharing
# the one GPU, no profiler (s3_2 under rocprofv3 had every candidate time out), IPC candidates.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
GPU_MAX_HW_QUEUES=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29652 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "row/default/ipc/kernel,row/default/ipc/kernel/blas,row/coll_pipeline/ipc/kernel/s4,row/p2p_pipeline/ipc/memcpy" > gpurun_out/s3_3_row2.log 2>&1; rc=$?
echo "row2 rc=$rc"; grep -a "\[bench\]" gpurun_out/s3_3_row2.log | cut -c1-160; tail -1 gpurun_out/s3_3_row2.log; exit $rc
