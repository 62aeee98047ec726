set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_1_tests.log 2>&1; rc=$?; tail -5 gpurun_out/s2_1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_1_smoke.log 2>&1 || { tail gpurun_out/s2_1_smoke.log; exit 1; }
tail -1 gpurun_out/s2_1_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s2_1_bench.log 2>&1 || { tail gpurun_out/s2_1_bench.log; exit 1; }
tail -1 gpurun_out/s2_1_bench.log
