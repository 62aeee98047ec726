# Round 2: persistent pt4 GEMM with arrival flags (CU reserve): GPU suite, fused rehearsal, N=1 bench
# then the ungated flagship at N=1 (regression check of the pt4 change)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 700 --timeout-method thread > gpurun_out/r2/r2_25_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r2/r2_25_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" gpurun_out/r2/r2_25_tests.log | tail -20; exit $rc; }
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/memcpy/s8/fused/graph,coll_pipeline/ipc/memcpy/s4/fused/graph,coll_pipeline/ipc/memcpy/s8/fused,coll_pipeline/ipc/memcpy/s8/graph"
start=$(date +%s)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/r2/r2_25_bench2.log 2>&1; rc=$?
echo "2 ranks rc=$rc wall=$(( $(date +%s) - start ))s"
grep -a "\[bench\]\|^{" gpurun_out/r2/r2_25_bench2.log | cut -c1-220
[ $rc -eq 0 ] || exit $rc
unset DDLB_ALLOW_SHARED_GPU DDLB_PG_BACKEND
timeout -k 10 300 python bench.py > gpurun_out/r2/r2_25_bench1.log 2>&1; rc=$?
grep -a "\[bench\]" gpurun_out/r2/r2_25_bench1.log; tail -1 gpurun_out/r2/r2_25_bench1.log | cut -c1-300; exit $rc
