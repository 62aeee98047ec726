set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread -k "rccl_data_plane" > gpurun_out/s2_13_tests.log 2>&1; rc=$?; tail -30 gpurun_out/s2_13_tests.log; exit $rc
