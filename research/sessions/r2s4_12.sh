# IPC configs incl. MX-fp8 in-kernel all-gather and MX-fp8 rowwise direct store (2-4 ranks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -k "ipc_shared" -x -v --timeout 500 --timeout-method thread > $O/ipc_tests.log 2>&1; rc=$?; tail -5 $O/ipc_tests.log; [ $rc -eq 0 ] || { grep -a "FAIL\|Error\|error" $O/ipc_tests.log | tail -30; exit $rc; }
