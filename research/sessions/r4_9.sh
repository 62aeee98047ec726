# round 4 / 9: shared-GPU rehearsals of the N>1 path: preflight with the new primitive phases
# (2 and 4 ranks on one GPU; RCCL refuses two ranks per device, so its phases fail there), then
# bench.py --gpus 2 over the leading candidates (col) and the direct-store rowwise
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_9
mkdir -p $O
export TMPDIR=/tmp DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 4 --preflight-only > $O/preflight4.log 2>&1; rc=$?
grep -a "\[bench\|preflight" $O/preflight4.log | cut -c1-400; [ $rc -le 1 ] || exit $rc
C="coll_pipeline/rccl/s4/fused,coll_pipeline/ipc/agk32/s4/graph,direct/ipc,coll_pipeline/ipc/agk32/s8/graph,default/ipc/kernel"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 2 --steps 20 --warmup 5 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2.log | cut -c1-250; grep -a metric $O/bench2.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
R="row/p2p_pipeline/ipc/direct/graph,row/default/ipc/kernel,row/p2p_pipeline/ipc/direct"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29721 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 20 --warmup 5 --candidates "$R" > $O/bench2_row.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2_row.log | cut -c1-250; grep -a metric $O/bench2_row.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc
