# direct-store C (c_shards, tile_order 2): world-1 GEMM test, whole GPU suite (IPC row/p2p/direct at
# 2-3 ranks), 2-rank shared-GPU rehearsal of the tp_rowwise config #3 shape, N=1 flagship bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -k "direct_store" -x -v --timeout 120 --timeout-method thread > $O/ds_tests.log 2>&1; rc=$?; tail -6 $O/ds_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" $O/gpu_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench\]" $O/bench.log; grep metric $O/bench.log | cut -c1-400
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="row/p2p_pipeline/ipc/direct/graph,row/p2p_pipeline/ipc/direct,row/p2p_pipeline/ipc/memcpy/graph,row/p2p_pipeline/ipc/memcpy,row/default/ipc/kernel,row/coll_pipeline/ipc/kernel/s4/graph"
start=$(date +%s)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --steps 10 --warmup 3 --candidates "$C" > $O/bench2_row.log 2>&1; rc=$?
echo "2 ranks rowwise rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" $O/bench2_row.log | cut -c1-260
exit $rc
