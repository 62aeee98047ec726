# Triage of the memcpy-protocol timeouts with 4 ranks on one GPU: fewer HW queues per process,
# and a small shape with the default queue count.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="p2p_pipeline/ipc/memcpy,coll_pipeline/ipc/memcpy/s4"
run() {  # tag, extra args
  tag=$1; shift
  start=$(date +%s)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --steps 10 --warmup 3 --candidate-timeout 40 --candidates "$C" "$@" > gpurun_out/s2_8_$tag.log 2>&1; rc=$?
  echo "$tag rc=$rc wall=$(( $(date +%s) - start ))s"
  grep -a "\[bench\]" gpurun_out/s2_8_$tag.log | cut -c1-200
}
GPU_MAX_HW_QUEUES=2 run q2
run small -m 4096
run q4
