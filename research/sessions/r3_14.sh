# world-1 capture topologies: which one crashes hipStreamEndCapture
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_14
mkdir -p $O
DDLB_GRAPH_DEBUG=1 timeout -k 10 300 python -u scripts/diag_graph_edges.py 2>&1 | tee $O/edges.txt
exit 0
