# Round 2: graph-captured signal plans — full GPU suite (IPC configs with graph=True at world
# 2-3), then the host enqueue cost per run of IPC plans with / without the graph (2 ranks).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 700 --timeout-method thread > gpurun_out/r2/r2_15_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2/r2_15_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" gpurun_out/r2/r2_15_tests.log | tail -20; exit $rc; }
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
for g in "" "--graph"; do
  for alg in "coll_pipeline -s 8" "coll_pipeline -s 8 --protocol kernel" "p2p_pipeline"; do
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29591 -m ddlb_amd.parallel.explain -m 65536 -n 1024 -k 1024 --timeline --backend ipc --algorithm $alg $g > gpurun_out/r2/r2_15_host.txt 2>&1 || { echo "failed: $alg $g"; tail -5 gpurun_out/r2/r2_15_host.txt; exit 1; }
    grep -a "host enqueue per run" gpurun_out/r2/r2_15_host.txt | head -1
  done
done
