# round 4 / 10: RCCL-fed fused plans with the signal kernels on their own stream (budget + timelines)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_10
mkdir -p $O
export TMPDIR=/tmp
TL="coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8/fused,p2p_pipeline/rccl/fused,coll_pipeline/rccl/s4,default/rccl"
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --timeline "coll_pipeline/rccl/s8/fused,p2p_pipeline/rccl/fused" --out $O/col8.json > $O/col8.txt 2>&1 || { echo "col8 failed"; tail -20 $O/col8.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|amdgpu.ids\|socket.cpp" $O/col8.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py -k "rccl" > $O/native.txt 2>&1 || { echo "native rccl tests failed"; tail -30 $O/native.txt; exit 1; }
tail -n 1 $O/native.txt
