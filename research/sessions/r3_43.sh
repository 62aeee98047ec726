# Rebuilt in-tree .so (comment-only source change): GEMM suite, native GPU suite, smoke, bench N=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_43
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; grep -a "FAILED\|Timeout" $O/gpu_tests.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a metric $O/bench.log | cut -c1-300
