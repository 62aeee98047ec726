# Full GPU suite (verbose: the name of a test that stalls is in the log), smoke, N=1 bench,
# 2-rank shared-GPU rehearsal with the preflight
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 170 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error\|Timeout" $O/gpu_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench" $O/bench.log; grep metric $O/bench.log | cut -c1-400
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/batch/s8/graph,direct/ipc,coll_pipeline/rccl/s4"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --steps 20 --warmup 5 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2.log | cut -c1-250; grep -a metric $O/bench2.log | cut -c1-600; exit $rc
