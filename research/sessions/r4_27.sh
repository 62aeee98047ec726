# round 4 / 27: 4 ranks sharing one GPU run ~20x slower than in round 2: hardware-queue
# oversubscription? Same candidates with GPU_MAX_HW_QUEUES 4 (default) and 2 per process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_27
mkdir -p $O
export TMPDIR=/tmp DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="direct/ipc,coll_pipeline/ipc/push/s4,default/ipc/kernel"
for q in 4 2; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2975$q bench.py --gpus 4 --steps 10 --warmup 3 --candidates "$C" --deadline-s 280 > $O/q$q.log 2>&1; rc=$?
  echo "== GPU_MAX_HW_QUEUES=$q"; grep -a "tune\|final\|preflight_ipc" $O/q$q.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
