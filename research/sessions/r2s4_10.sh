# A/B of the hipGraph prologue fusion in one call (same box): agk world 1, 2-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_10
mkdir -p $O
F="amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|destroy_process_group"
for v in 0 1 0 1; do
  DDLB_GRAPH_PROLOGUE=$v timeout -k 10 300 python -u scripts/bench_agk_world1.py --ctas 32 --modes 14,14 --iters 200 > $O/agk_world1_p$v.log 2>&1; rc=$?; echo "prologue=$v"; grep -v "$F" $O/agk_world1_p$v.log | tail -3; [ $rc -eq 0 ] || exit $rc
done
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk32/s4/graph"
for v in 0 1; do
  DDLB_GRAPH_PROLOGUE=$v timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2959$v bench.py --gpus 2 --steps 50 --warmup 5 --tune-rounds 2 --candidates "$C" > $O/bench2_p$v.log 2>&1; rc=$?
  echo "prologue=$v"; grep -a "\[bench\]" $O/bench2_p$v.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
