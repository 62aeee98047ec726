set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g16_tests.log 2>&1; rc=$?; tail -5 gpurun_out/g16_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/g16_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/g16_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/g16_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/g16_bench.log; exit 1; }
grep metric gpurun_out/g16_bench.log
timeout -k 10 300 python scripts/diag_bench_gap.py > gpurun_out/g16_gap.log 2>&1; grep -v "amdgpu.ids\|^\[W" gpurun_out/g16_gap.log | tail -8
