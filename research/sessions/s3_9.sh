# Session 3: copy kernel back on plain loads (default), A/B again, full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_reduce.py --copy > gpurun_out/s3_9_copy.txt 2>&1 || exit 5
DDLB_COPY_NT=1 timeout -k 10 120 python scripts/bench_reduce.py --copy >> gpurun_out/s3_9_copy.txt 2>&1 || exit 6
timeout -k 10 120 python scripts/bench_reduce.py --copy >> gpurun_out/s3_9_copy.txt 2>&1 || exit 7
grep copy gpurun_out/s3_9_copy.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_9_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s3_9_tests.log; exit $rc
