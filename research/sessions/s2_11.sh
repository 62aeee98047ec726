set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 300 --timeout-method thread -k "ipc_shared" > gpurun_out/s2_11_tests.log 2>&1; rc=$?; tail -4 gpurun_out/s2_11_tests.log; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="p2p_pipeline/ipc/push,p2p_pipeline/ipc/push/blas,default/ipc/push,coll_pipeline/ipc/push/s4,default/ipc/kernel/push,p2p_pipeline/ipc/memcpy"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_11_bench2.log 2>&1; rc=$?
echo "n=2 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_11_bench2.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 8 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_11_bench8.log 2>&1; rc=$?
echo "n=8 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_11_bench8.log | cut -c1-200; exit $rc
