set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_23_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s2_23_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_23_smoke.log 2>&1 || { tail gpurun_out/s2_23_smoke.log; exit 1; }
tail -1 gpurun_out/s2_23_smoke.log
timeout -k 10 300 python scripts/diag_blas_tune.py > gpurun_out/s2_23_tune.log 2>&1 || { tail gpurun_out/s2_23_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s2_23_tune.log
for dt in bfloat16 float8_e4m3fn; do
  timeout -k 10 300 python bench.py --dtype $dt > gpurun_out/s2_23_bench_$dt.log 2>&1 || { tail gpurun_out/s2_23_bench_$dt.log; exit 1; }
  grep -ao '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"algorithm": "[^"]*"\|"autotune_ms.*' gpurun_out/s2_23_bench_$dt.log | tr '\n' ' '; echo
done
