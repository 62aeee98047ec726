# Round 2: IPC shared-GPU tests incl. copy_streams=2 (memcpy pulls over 2 copy streams per peer)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py -x -v -m gpu -k "ipc_shared" --timeout 700 --timeout-method thread > gpurun_out/r2/r2_21.log 2>&1; rc=$?
grep -a "PASS\|FAIL\|Error" gpurun_out/r2/r2_21.log | tail -8; exit $rc
