# Round 2: RCCL collectives inside a captured plan graph (world 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -v -m gpu -k "rccl_data_plane or timeline or capturable" --timeout 120 --timeout-method thread > gpurun_out/r2/r2_19.log 2>&1; rc=$?
grep -a "PASS\|FAIL\|Error" gpurun_out/r2/r2_19.log | tail -8; exit $rc
