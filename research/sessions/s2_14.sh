set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/s2_14_col.log 2>&1 || { tail gpurun_out/s2_14_col.log; exit 1; }
grep -a "^{" gpurun_out/s2_14_col.log | cut -c1-700
timeout -k 10 300 python bench.py --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > gpurun_out/s2_14_row.log 2>&1 || { tail gpurun_out/s2_14_row.log; exit 1; }
grep -a "^{" gpurun_out/s2_14_row.log | cut -c1-900
timeout -k 10 300 python bench.py --dtype float8_e4m3fn > gpurun_out/s2_14_fp8.log 2>&1 || { tail gpurun_out/s2_14_fp8.log; exit 1; }
grep -a "^{" gpurun_out/s2_14_fp8.log | cut -c1-900
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="row/default/ipc/kernel,row/default/ipc/kernel/blas,row/coll_pipeline/ipc/kernel/s4,row/p2p_pipeline/ipc/memcpy"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29601 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/s2_14_row2.log 2>&1; rc=$?
echo "row n=2 rc=$rc"; grep -a "\[bench\]\|^{" gpurun_out/s2_14_row2.log | cut -c1-300; exit $rc
