# 4- and 8-rank shared-GPU rehearsals of the in-kernel all-gather candidates (single-stream
# plans: no copy-stream HW-queue pressure); interleaved copy units over 3 / 7 producers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_4
mkdir -p $O
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk32/s8,coll_pipeline/ipc/agk64/s8/graph"
for n in 4 8; do
  start=$(date +%s)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2956$n bench.py --gpus $n --steps 10 --warmup 3 --candidates "$C" > $O/bench$n.log 2>&1; rc=$?
  echo "$n ranks rc=$rc wall=$(( $(date +%s) - start ))s"
  grep -a "\[bench\]\|^{" $O/bench$n.log | cut -c1-220
  [ $rc -eq 0 ] || exit $rc
done
