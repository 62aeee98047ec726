# round 4 / 2: one-GPU per-rank budget (EMULATED) of every N>1 candidate at d = 8: BASELINE
# configs #4 (columnwise bf16), #3 (rowwise), #5 dtype (fp8); rocprofv3 kernel stats of the
# config-#4 winners
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/gemm.txt 2>&1 || { echo "gemm tests failed"; tail -30 $O/gemm.txt; exit 1; }
tail -n 2 $O/gemm.txt
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_native_gpu.py -k "cu_split or rccl_data_plane or a_table or rccl_fed" > $O/native.txt 2>&1 || { echo "native tests failed"; tail -30 $O/native.txt; exit 1; }
tail -n 2 $O/native.txt
grep "cu-masked" $O/native.txt | head -3
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --out $O/col8.json > $O/col8.txt 2>&1 || { echo "col8 failed"; tail -20 $O/col8.txt; exit 1; }
cat $O/col8.txt
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 --out $O/row8.json > $O/row8.txt 2>&1 || { echo "row8 failed"; tail -20 $O/row8.txt; exit 1; }
cat $O/row8.txt
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --dtype float8_e4m3fn --out $O/fp8_8.json > $O/fp8_8.txt 2>&1 || { echo "fp8 failed"; tail -20 $O/fp8_8.txt; exit 1; }
cat $O/fp8_8.txt
