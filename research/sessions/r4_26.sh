# round 4 / 26: whole N>1 pools rehearsed with ranks sharing the GPU (IPC families; RCCL refuses
# two ranks per device): 4-rank columnwise, 2-rank rowwise; N=1 rowwise config #3 shape and fp8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_26
mkdir -p $O
export TMPDIR=/tmp DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29741 bench.py --gpus 4 --steps 10 --warmup 3 --deadline-s 500 > $O/bench4_col.log 2>&1; rc=$?
grep -a "\[bench" $O/bench4_col.log | cut -c1-220; grep -a '^{' $O/bench4_col.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29743 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --deadline-s 500 > $O/bench2_row.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2_row.log | cut -c1-220; grep -a '^{' $O/bench2_row.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
