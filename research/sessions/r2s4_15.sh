# Whole N>1 pools rehearsed with 2 ranks sharing the GPU (every IPC candidate must validate;
# RCCL candidates fail fast: RCCL refuses two ranks per device)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_15
mkdir -p $O
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
start=$(date +%s)
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 10 --warmup 3 --candidate-timeout 45 > $O/bench2_col_full.log 2>&1; rc=$?
echo "col rc=$rc wall=$(( $(date +%s) - start ))s"; grep -a "\[bench\]" $O/bench2_col_full.log | cut -c1-160; grep -a "^{" $O/bench2_col_full.log | cut -c1-200
start=$(date +%s)
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --candidate-timeout 45 > $O/bench2_row_full.log 2>&1; rc2=$?
echo "row rc=$rc2 wall=$(( $(date +%s) - start ))s"; grep -a "\[bench\]" $O/bench2_row_full.log | cut -c1-160; grep -a "^{" $O/bench2_row_full.log | cut -c1-200
[ $rc -eq 0 ] && [ $rc2 -eq 0 ]
