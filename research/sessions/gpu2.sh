set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/g2_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g2_smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/g2_bench_native.log 2>&1 || exit 4
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --impl pytorch > gpurun_out/g2_bench_pytorch.log 2>&1 || exit 5
tail -1 gpurun_out/g2_bench_native.log; tail -1 gpurun_out/g2_bench_pytorch.log
