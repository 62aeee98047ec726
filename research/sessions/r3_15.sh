# capture-topology diagnostics after the executor fix (wait-only streams not joined), then the real 2-rank cs2 graph pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_15
mkdir -p $O
timeout -k 10 300 python -u scripts/diag_graph_edges.py 2>&1 | tee $O/edges.txt
CFG='[["col/coll_pipeline/memcpy/cs2/graph", "col", {"algorithm": "coll_pipeline", "backend": "ipc", "s": 2, "copy_streams": 2, "graph": true}], ["col/p2p_pipeline/memcpy/cs2/graph", "col", {"algorithm": "p2p_pipeline", "backend": "ipc", "copy_streams": 2, "graph": true}], ["row/coll_pipeline/memcpy/cs2/graph", "row", {"algorithm": "coll_pipeline", "backend": "ipc", "copy_streams": 2, "graph": true}]]'
PORT=29681
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_GRAPH_CS2=1 \
  DDLB_TEST_CFGS="$CFG" timeout -k 10 150 python3 -u tests/_ipc_worker.py > $O/rank$r.log 2>&1 &
done
wait
tail -8 $O/rank0.log; tail -8 $O/rank1.log
exit 0
