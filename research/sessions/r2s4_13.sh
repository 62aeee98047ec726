# fp8 (BASELINE config #5 dtype) N>1 rehearsal: 2 ranks sharing a GPU, agk / memcpy candidates, MX
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_13
mkdir -p $O
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk32/s8/graph/mx,coll_pipeline/ipc/agk32/s4/graph/mx,coll_pipeline/ipc/memcpy/s8/graph/mx,p2p_pipeline/ipc/memcpy/graph/mx"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dtype float8_e4m3fn --steps 50 --warmup 5 --candidates "$C" > $O/bench2_fp8.log 2>&1; rc=$?
grep -a "\[bench\]\|^{" $O/bench2_fp8.log | cut -c1-220; exit $rc
