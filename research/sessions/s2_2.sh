set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
start=$(date +%s)
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --candidate-timeout 60 > gpurun_out/s2_2_bench2.log 2>&1; rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start ))s"
grep -v amdgpu.ids gpurun_out/s2_2_bench2.log | grep -v "socket.cpp\|Gloo\|version\|Hostname\|Librccl" | tail -30
