# Round 2: full GPU suite after the time-ordered enqueue of the IPC pulls (world 2-4 shared-GPU
# IPC tests run with one HW queue per process at world 4: every stream shares one queue).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 700 --timeout-method thread > gpurun_out/r2/r2_10_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2/r2_10_tests.log; exit $rc
