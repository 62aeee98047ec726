# 2 ranks sharing the one GPU (gloo control plane, IPC data plane): the CLI runner at larger
# shapes, every IPC algorithm of both primitives, reference timing modes, validation.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
IMPLS_COL=(--impl "native;algorithm=default,coll_pipeline,p2p_pipeline;backend=ipc;multicast_protocol=memcpy,kernel;s=4" --impl "native;algorithm=direct;backend=ipc" --impl "native;algorithm=p2p_pipeline;backend=ipc;fused" --impl "native;algorithm=default,coll_pipeline;backend=ipc;order=AG_after;s=4" --impl "native;algorithm=default,p2p_pipeline;backend=ipc;gemm_mode=blas")
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 -m ddlb_amd --primitive tp_columnwise -m 16384 -n 1024 -k 1024 --dtype bfloat16 --num-iterations 20 --num-warmups 5 --child-timeout 90 --output-csv gpurun_out/s2_5_col.csv "${IMPLS_COL[@]}" > gpurun_out/s2_5_col.log 2>&1; rc=$?
echo "col rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 -m ddlb_amd --primitive tp_rowwise -m 8192 -n 4096 -k 4096 --dtype bfloat16 --num-iterations 20 --num-warmups 5 --child-timeout 90 --time-measurement-backend cuda_event --output-csv gpurun_out/s2_5_row.csv --impl "native;algorithm=default,coll_pipeline,p2p_pipeline;backend=ipc;multicast_protocol=memcpy,kernel;s=4" > gpurun_out/s2_5_row.log 2>&1; rc=$?
echo "row rc=$rc"; exit $rc
