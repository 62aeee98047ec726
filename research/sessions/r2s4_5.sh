# AG_FILL_ROUNDS (ag_mode 8): copy workgroups grown while the GEMM's tile rounds stay the same
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_5
mkdir -p $O
F="amdgpu.ids\|socket.cpp\|^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|destroy_process_group"
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -k "in_kernel_allgather or flag_gated" -x -q --timeout 120 --timeout-method thread > $O/agk_tests.log 2>&1; rc=$?; tail -2 $O/agk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_agk_world1.py --ctas 32 --modes 6,14,6,14,0,8 --iters 100 > $O/agk_world1.log 2>&1; rc=$?; grep -v "$F" $O/agk_world1.log | tail -12; [ $rc -eq 0 ] || exit $rc
