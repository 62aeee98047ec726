# Full GPU suite + smoke on the final kernels; kernel trace of the in-kernel all-gather (world 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_8
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" $O/gpu_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_agk -- python scripts/bench_agk_world1.py --ctas 32 --modes 14 --iters 50 > $O/prof_agk.log 2>&1; echo "prof rc=$?"
find $O/prof_agk -name "*kernel_stats.csv" | head -3
