# Session 3: BASELINE config #3 shape (tp_rowwise GEMM + reduce-scatter, m=16384 n=8192 k=8192 bf16)
# at N=1, then 2 ranks sharing the one GPU (gloo control group, every IPC candidate) under
# rocprofv3 --kernel-trace --stats for the per-kernel split (GEMM vs fused d-way reduce / copies).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 20 --warmup 5 > gpurun_out/s3_2_row_n1.log 2>&1; rc=$?
echo "row n1 rc=$rc"; tail -1 gpurun_out/s3_2_row_n1.log; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
GPU_MAX_HW_QUEUES=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_2_prof -o row2 -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 > gpurun_out/s3_2_row2.log 2>&1; rc=$?
echo "row2 rc=$rc"; grep -a "\[bench\]" gpurun_out/s3_2_row2.log | cut -c1-160; tail -1 gpurun_out/s3_2_row2.log; exit $rc
