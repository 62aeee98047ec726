set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_10_tests.log 2>&1; rc=$?; tail -15 gpurun_out/s2_10_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_10_smoke.log 2>&1 || { tail gpurun_out/s2_10_smoke.log; exit 1; }
tail -1 gpurun_out/s2_10_smoke.log
