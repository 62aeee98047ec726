set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/g13_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/g13_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/g13_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/g13_bench.log; exit 1; }
grep metric gpurun_out/g13_bench.log
timeout -k 10 300 python bench.py --algorithm "pytorch(rccl+hipblaslt)" > gpurun_out/g13_bench_pt.log 2>&1 || { echo bench pt failed; exit 1; }
grep metric gpurun_out/g13_bench_pt.log
timeout -k 10 300 python scripts/bench_gemm.py --tiles auto,i256,pi256,128x128 --shapes all --json gpurun_out/g13_gemm_bf16.json > gpurun_out/g13_gemm_bf16.log 2>&1; echo "gemm rc=$?"
