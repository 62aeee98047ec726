# AG_WAIT_ACKS (the launch waits for the peers' ACKs; no wait kernel after it): tests + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_14
mkdir -p $O
F="amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|destroy_process_group"
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -a "FAIL\|Error" $O/tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -u scripts/bench_agk_world1.py --ctas 32 --modes 14,30,14,30 --iters 200 > $O/agk_world1.log 2>&1; rc=$?; grep -v "$F" $O/agk_world1.log | tail -5; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk32/s4/graph"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 50 --warmup 5 --tune-rounds 2 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench\]" $O/bench2.log | cut -c1-200; exit $rc
