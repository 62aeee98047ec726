# round 4 / 25: pt4 from 128 tiles up: GPU suite, budget of the stage-GEMM plans, bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_25
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
TL="coll_pipeline/rccl/s8,coll_pipeline/rccl/s4,p2p_pipeline/rccl,coll_pipeline/ipc/memcpy/s8/graph,coll_pipeline/rccl/s4/fused"
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --candidates "$TL" > $O/col8.txt 2>&1 || { echo "budget failed"; tail -20 $O/col8.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp" $O/col8.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
