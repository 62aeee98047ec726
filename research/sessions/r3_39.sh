# Validation of the VALU-free pt4 product: GPU suite, smoke, N=1 bench, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_39
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 170 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -4 $O/gpu_tests.log; grep -a "FAILED\|Timeout" $O/gpu_tests.log | tail -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench" $O/bench.log | cut -c1-200; grep metric $O/bench.log | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python bench.py --steps 50 --warmup 5 > $O/prof_bench.log 2>&1; echo "prof rc=$?"
find $O/prof -name "*kernel_stats.csv" | head -3
export DDLB_ALLOW_SHARED_GPU=1
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench2.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2.log | cut -c1-250; grep -a metric $O/bench2.log | cut -c1-900; exit $rc
