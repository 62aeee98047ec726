# bench.py with 4 and 8 ranks sharing the one GPU (gloo control plane, IPC candidates only:
# RCCL refuses duplicate devices). Timings are meaningless here; this checks the d=4/d=8
# protocols (flags, per-peer streams, shard tables) and the orchestration at the flagship shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="direct/ipc,p2p_pipeline/ipc/memcpy,p2p_pipeline/ipc/memcpy/blas,p2p_pipeline/ipc/memcpy/fused,coll_pipeline/ipc/memcpy/s4,default/ipc/kernel,default/ipc/kernel/blas"
for n in 4 8; do
  start=$(date +%s)
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2955$n bench.py --gpus $n --steps 10 --warmup 3 --candidate-timeout 90 --candidates "$C" > gpurun_out/s2_7_bench$n.log 2>&1; rc=$?
  echo "n=$n rc=$rc wall=$(( $(date +%s) - start ))s"
  grep -a "\[bench\]\|^{" gpurun_out/s2_7_bench$n.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
