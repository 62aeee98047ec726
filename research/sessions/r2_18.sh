# Round 2: bench.py full N>1 pool with 2 ranks sharing the GPU (validated tuning, graph candidates)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
start=$(date +%s)
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --candidate-timeout 60 > gpurun_out/r2/r2_18_bench2.log 2>&1; rc=$?
echo "2 ranks rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" gpurun_out/r2/r2_18_bench2.log | cut -c1-220
exit $rc
