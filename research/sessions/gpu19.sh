set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g19_tests.log 2>&1; rc=$?; tail -15 gpurun_out/g19_tests.log; [ $rc -eq 0 ] || exit $rc
