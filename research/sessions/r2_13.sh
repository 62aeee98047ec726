# Round 2: per-op host enqueue cost of the IPC coll_pipeline plan (4 ranks sharing the GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo GPU_MAX_HW_QUEUES=2
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29591 -m ddlb_amd.parallel.explain -m 65536 -n 1024 -k 1024 --timeline --algorithm coll_pipeline --backend ipc -s 8 > gpurun_out/r2/r2_13_coll_memcpy_s8_d4.txt 2>&1; rc=$?
grep -a "host enqueue\|rank 0" gpurun_out/r2/r2_13_coll_memcpy_s8_d4.txt | head -4
awk '/rank 0\/4/{p=1} /rank 1\/4/{p=0} p' gpurun_out/r2/r2_13_coll_memcpy_s8_d4.txt | head -70
exit $rc
