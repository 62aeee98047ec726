# round 4 / 1: pt4 on grouped-row and table A, the RCCL-fed gated GEMM (world-1 forms), then the
# flagship bench at N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_native_gpu.py -k "a_table or rccl_fed or rccl_fused or flag_gated or in_kernel or direct_store or native_world1" \
  > $O/native.txt 2>&1 || { echo "native tests failed"; tail -30 $O/native.txt; exit 1; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "grouped or pt4 or t8_kernel or long_k" \
  > $O/gemm.txt 2>&1 || { echo "gemm tests failed"; tail -30 $O/gemm.txt; exit 1; }
tail -3 $O/native.txt $O/gemm.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
cat $O/bench.json | cut -c1-600
