# Session 3: re-verification after the container rebuild (fresh in-tree .so): GPU suite, smoke, N=1 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_1_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s3_1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_1_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/s3_1_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s3_1_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 gpurun_out/s3_1_bench.log; exit $rc
