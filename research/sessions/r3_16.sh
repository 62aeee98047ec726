# side-stream cycle guard + cs2 graph pipelines in the IPC shared-GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_16
mkdir -p $O
timeout -k 10 300 python -u scripts/diag_graph_edges.py > $O/edges.txt 2>&1; cat $O/edges.txt
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "cycle or ipc_shared_gpu or graph" > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; grep -a "FAILED\|Timeout\|Error" $O/tests.log | head -20; exit $rc
