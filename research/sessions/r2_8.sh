# Round 2: plan timeline (per-op GPU timing events) — GPU test, then the timeline of the world-1
# flagship coll_pipeline plan and of a 2-rank shared-GPU IPC coll_pipeline plan.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q -m gpu -k "timeline or world1" --timeout 120 --timeout-method thread > gpurun_out/r2/r2_8_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r2/r2_8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -m ddlb_amd.parallel.explain -m 65536 -n 1024 -k 1024 --algorithm default --backend rccl --timeline > gpurun_out/r2/r2_8_timeline_w1.txt 2>&1; rc=$?
cat gpurun_out/r2/r2_8_timeline_w1.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 -m ddlb_amd.parallel.explain -m 65536 -n 1024 -k 1024 --algorithm coll_pipeline --backend ipc -s 4 --timeline > gpurun_out/r2/r2_8_timeline_2rank.txt 2>&1; rc=$?
grep -v "amdgpu.ids\|W1016\|socket.cpp" gpurun_out/r2/r2_8_timeline_2rank.txt | head -60; exit $rc
