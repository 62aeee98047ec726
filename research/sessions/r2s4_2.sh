set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_2
mkdir -p $O
# in-kernel all-gather variants first (new copy-role publication), then the whole suite
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -k "in_kernel_allgather or flag_gated" -x -v --timeout 120 --timeout-method thread > $O/agk_tests.log 2>&1; rc=$?; tail -3 $O/agk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_agk_world1.py --ctas 32,64 --modes 1,0,2,4,6 --iters 50 > $O/agk_world1.log 2>&1; rc=$?; grep -v "amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/agk_world1.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep metric $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python bench.py --steps 50 --algorithm "gemm (world=1)/hip" > $O/prof.log 2>&1; echo "prof rc=$?"
find $O/prof -name "*kernel_stats.csv" | head
