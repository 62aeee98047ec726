# pt4 epilogue after c_row (global-address-space C pointers): flagship bench N=1, GEMM shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_7
mkdir -p $O
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench\]" $O/bench.log; grep metric $O/bench.log | cut -c1-300
timeout -k 10 300 python scripts/bench_gemm.py --rounds 3 --iters 20 --tiles auto,t4 --modes auto,blas --shapes 0,1,2 > $O/gemm.log 2>&1; rc=$?; grep -v "amdgpu.ids\|socket.cpp" $O/gemm.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; exit $rc
