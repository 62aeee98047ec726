# Full GPU suite, smoke, N=1 bench, 2-rank rehearsal; then the cs2 graph crash backtrace and a per-stage roctx trace
# 2-rank shared-GPU rehearsal with the preflight
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 170 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -4 $O/gpu_tests.log; grep -a "FAILED\|Timeout" $O/gpu_tests.log | tail -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench" $O/bench.log; grep metric $O/bench.log | cut -c1-400
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/agk32/s8/graph,coll_pipeline/ipc/batch/s8/graph,direct/ipc,coll_pipeline/rccl/s4"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --steps 20 --warmup 5 --candidates "$C" > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2.log | cut -c1-250; grep -a metric $O/bench2.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc

CFG='[["col/coll_pipeline/memcpy/cs2/graph", "col", {"algorithm": "coll_pipeline", "backend": "ipc", "s": 2, "copy_streams": 2, "graph": true}]]'
PORT=29661
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_CRASH_BT=1 DDLB_GRAPH_CS2=1 \
  DDLB_TEST_CFGS="$CFG" timeout -k 10 100 python -u tests/_ipc_worker.py > $O/cs2_graph_rank$r.log 2>&1 &
done
wait
tail -40 $O/cs2_graph_rank0.log; tail -40 $O/cs2_graph_rank1.log
PORT=29663
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 \
  timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --kernel-rename --stats -d $O/trace_r$r -o tr -- python3 scripts/trace_pipeline.py --algorithm coll_pipeline --backend ipc -s 4 > $O/trace_rank$r.log 2>&1 &
done
wait
tail -3 $O/trace_rank0.log
