set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
start=$(date +%s)
( export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo; timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --candidate-timeout 60 > gpurun_out/s2_3_bench2.log 2>&1 ); rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" gpurun_out/s2_3_bench2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python scripts/diag_blas_batch.py > gpurun_out/s2_3_blas.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/s2_3_blas.log | tail -30; exit $rc
