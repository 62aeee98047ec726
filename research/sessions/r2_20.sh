# Round 2 checkpoint: full GPU suite, smoke, N=1 bench on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 700 --timeout-method thread > gpurun_out/r2/r2_20_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r2/r2_20_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" gpurun_out/r2/r2_20_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/r2_20_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r2/r2_20_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r2/r2_20_bench.log 2>&1; rc=$?
tail -1 gpurun_out/r2/r2_20_bench.log | cut -c1-400; exit $rc
