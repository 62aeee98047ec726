set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_12_tests.log 2>&1; rc=$?; tail -6 gpurun_out/s2_12_tests.log; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo GPU_MAX_HW_QUEUES=1
C="default/ipc/kernel,default/ipc/kernel/push,p2p_pipeline/ipc/memcpy"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 8 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_12_bench8.log 2>&1; rc=$?
echo "n=8 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_12_bench8.log | cut -c1-200; exit $rc
