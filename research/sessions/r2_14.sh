# Round 2: hipGraph branch concurrency check
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 120 python scripts/diag_graph_concurrency.py > gpurun_out/r2/r2_14_graph.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r2/r2_14_graph.txt; exit $rc
