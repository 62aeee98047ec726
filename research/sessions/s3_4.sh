# Session 3: per-kernel split of tp_rowwise (config #3 shape) with 2 ranks sharing the GPU, IPC
# candidates only (no RCCL child that fails on a shared device), under rocprofv3 kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_4_prof -o row2 --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29653 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "row/default/ipc/kernel,row/p2p_pipeline/ipc/memcpy" > gpurun_out/s3_4_row2.log 2>&1; rc=$?
echo "row2 prof rc=$rc"; grep -a "\[bench\]" gpurun_out/s3_4_row2.log | cut -c1-160; find gpurun_out/s3_4_prof -name "*stats*" | head; exit $rc
