set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g18_tests.log 2>&1; rc=$?; tail -5 gpurun_out/g18_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/g18_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/g18_bench.log; exit 1; }
grep metric gpurun_out/g18_bench.log
timeout -k 10 400 python bench.py --warmup 5 --steps 20 > gpurun_out/g18_bench2.log 2>&1 || { echo bench2 failed; tail -20 gpurun_out/g18_bench2.log; exit 1; }
grep metric gpurun_out/g18_bench2.log
