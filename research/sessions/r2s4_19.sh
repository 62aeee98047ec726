# After the pt4 write-through C stores: full GPU suite, smoke, agk world 1, 2-rank rehearsal, N=1 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_19
mkdir -p $O
F="amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|destroy_process_group"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" $O/gpu_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u scripts/bench_agk_world1.py --ctas 32 --modes 30,30 --iters 200 > $O/agk_world1.log 2>&1; rc=$?; grep -v "$F" $O/agk_world1.log | tail -3; [ $rc -eq 0 ] || exit $rc
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/agk32/s4/graph,direct/ipc"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --steps 20 --warmup 5 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench\]" $O/bench2.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
unset DDLB_ALLOW_SHARED_GPU DDLB_PG_BACKEND
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench\]" $O/bench.log; grep metric $O/bench.log | cut -c1-250
