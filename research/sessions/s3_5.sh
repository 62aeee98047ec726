# Session 3: reduce kernel — numerics of every source count / dtype, A/B of the fixed-count
# unrolled kernels vs the runtime-count kernel on local HBM, then the rowwise 2-rank profile again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_reduce_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_5_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s3_5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bench_reduce.py > gpurun_out/s3_5_reduce_fixed.txt 2>&1 || exit 5
DDLB_REDUCE_GENERIC=1 timeout -k 10 120 python scripts/bench_reduce.py > gpurun_out/s3_5_reduce_generic.txt 2>&1 || exit 6
timeout -k 10 120 python scripts/bench_reduce.py >> gpurun_out/s3_5_reduce_fixed.txt 2>&1 || exit 7
cat gpurun_out/s3_5_reduce_*.txt
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_5_prof -o row2 --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29654 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "row/default/ipc/kernel,row/p2p_pipeline/ipc/memcpy" > gpurun_out/s3_5_row2.log 2>&1; rc=$?
echo "row2 prof rc=$rc"; grep -a "\[bench\]" gpurun_out/s3_5_row2.log | cut -c1-160; exit $rc
