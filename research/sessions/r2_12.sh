# Round 2: host enqueue cost per run() of the IPC plans (ranks sharing the GPU; GPU timings are
# meaningless here, the host-side numbers are what this measures).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo GPU_MAX_HW_QUEUES=2
run() {  # tag nranks args...
  tag=$1; n=$2; shift 2
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29591 -m ddlb_amd.parallel.explain -m 65536 -n 1024 -k 1024 --timeline "$@" > gpurun_out/r2/r2_12_$tag.txt 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/r2/r2_12_$tag.txt; return 1; }
  grep -a "host enqueue" gpurun_out/r2/r2_12_$tag.txt | head -1 | sed "s/^/$tag: /"
}
run coll_memcpy_s8_d4 4 --algorithm coll_pipeline --backend ipc -s 8 && \
run coll_memcpy_s8_d4_ksig 4 --algorithm coll_pipeline --backend ipc -s 8 --signal-method kernel && \
run coll_kernel_s8_d4 4 --algorithm coll_pipeline --backend ipc -s 8 --protocol kernel && \
run default_kernel_d4 4 --algorithm default --backend ipc --protocol kernel && \
run p2p_memcpy_d4 4 --algorithm p2p_pipeline --backend ipc && \
run direct_d4 4 --algorithm direct --backend ipc
