# Round 2: hipGraph replay of a 9-stream plan under 4 (default), 2 and 1 HW queues per process
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
for q in 4 2 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python scripts/diag_graph_streams.py > gpurun_out/r2/r2_17_q$q.txt 2>&1; rc=$?
  echo "queues=$q rc=$rc"; grep -v "amdgpu.ids\|socket.cpp" gpurun_out/r2/r2_17_q$q.txt | tail -2
done
