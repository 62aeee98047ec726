# hipGraph prologue: run-counter bump fused with the plan's leading signals (one launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_9
mkdir -p $O
F="amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|destroy_process_group"
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" $O/tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -u scripts/bench_agk_world1.py --ctas 32 --modes 14,14 --iters 100 > $O/agk_world1.log 2>&1; rc=$?; grep -v "$F" $O/agk_world1.log | tail -4; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk64/s8/graph,coll_pipeline/ipc/agk32/s4/graph,coll_pipeline/ipc/memcpy/s8/graph"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 --steps 20 --warmup 3 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench\]\|^{" $O/bench2.log | cut -c1-220
exit $rc
