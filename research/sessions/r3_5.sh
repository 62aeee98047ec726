# (1) native backtrace of the copy_streams=2 hipGraph replay crash, 2 ranks
# sharing the GPU, crash handler on; (2) per-stage roctx trace of a 2-rank IPC coll_pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_5
mkdir -p $O
CFG='[["col/coll_pipeline/memcpy/cs2/graph", "col", {"algorithm": "coll_pipeline", "backend": "ipc", "s": 2, "copy_streams": 2, "graph": true}]]'
PORT=29661
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_CRASH_BT=1 DDLB_GRAPH_CS2=1 \
  DDLB_TEST_CFGS="$CFG" timeout -k 10 100 python -u tests/_ipc_worker.py > $O/cs2_graph_rank$r.log 2>&1 &
done
wait
tail -40 $O/cs2_graph_rank0.log; tail -40 $O/cs2_graph_rank1.log
PORT=29663
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 \
  timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --kernel-rename --stats -d $O/trace_r$r -o tr -- python3 scripts/trace_pipeline.py --algorithm coll_pipeline --backend ipc -s 4 > $O/trace_rank$r.log 2>&1 &
done
wait
tail -3 $O/trace_rank0.log
