# Session 3: reduce kernel A/B after non-temporal loads/stores in the fixed-count kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_reduce_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_6_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s3_6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bench_reduce.py > gpurun_out/s3_6_reduce.txt 2>&1 || exit 5
DDLB_REDUCE_GENERIC=1 timeout -k 10 120 python scripts/bench_reduce.py >> gpurun_out/s3_6_reduce.txt 2>&1 || exit 6
timeout -k 10 120 python scripts/bench_reduce.py >> gpurun_out/s3_6_reduce.txt 2>&1 || exit 7
grep reduce gpurun_out/s3_6_reduce.txt
