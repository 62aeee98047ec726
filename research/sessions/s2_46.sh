# Full default autotune pool (incl. the kernel-signal hedges) with 4 ranks sharing the one GPU
# (one HW queue each), exactly as the driver launches N>1 apart from the shared device.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
GPU_MAX_HW_QUEUES=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29646 bench.py --gpus 4 --steps 10 --warmup 3 > gpurun_out/s2_46_b4.log 2>&1; rc=$?
echo "n=4 rc=$rc"; grep -a "\[bench\]" gpurun_out/s2_46_b4.log | cut -c1-150; grep -ao '"valid": [a-z]*\|"algorithm": "[^"]*"' gpurun_out/s2_46_b4.log; exit $rc
