# round 4 / 6: stream pool + home stream: stall diagnosis again, native GPU tests, budget
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_6
mkdir -p $O
export TMPDIR=/tmp
#timeout -k 10 300 python -u scripts/diag_side_stream_stall.py --variants base,prio0,private > $O/stall.txt 2>&1 || { echo "diag failed"; tail -20 $O/stall.txt; exit 1; }
#grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/stall.txt
timeout -k 10 300 python -u scripts/diag_side_stream_stall.py --candidate coll_pipeline/rccl/s4 --variants base,prio0 > $O/stall_s4.txt 2>&1 || { echo "diag s4 failed"; tail -20 $O/stall_s4.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/stall_s4.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py tests/test_reduce_gpu.py tests/test_cli_gpu.py > $O/native.txt 2>&1 || { echo "native tests failed"; tail -30 $O/native.txt; exit 1; }
tail -n 2 $O/native.txt
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --out $O/col8.json > $O/col8.txt 2>&1 || { echo "col8 failed"; tail -20 $O/col8.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/col8.txt
