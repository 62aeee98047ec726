# Round 2: ADVICE fixes (multi-shard arrival wait, uncached flag words, per-stream hipBLASLt
# workspaces + bind-time tuning, validated autotune): GPU suite, then N=1 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2/r2_2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r2/r2_2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r2/r2_2_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/r2/r2_2_bench.log; exit $rc
