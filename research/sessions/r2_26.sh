# Round 2: pt4 gated form as its own instantiation: GPU suite + N=1 flagship bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 700 --timeout-method thread > gpurun_out/r2/r2_26_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r2/r2_26_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" gpurun_out/r2/r2_26_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/r2/r2_26_bench1.log 2>&1; rc=$?
grep -a "\[bench\]" gpurun_out/r2/r2_26_bench1.log; tail -1 gpurun_out/r2/r2_26_bench1.log | cut -c1-300; exit $rc
