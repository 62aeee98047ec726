set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_native_gpu.py -x -q > gpurun_out/g3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/g3_tests.log
