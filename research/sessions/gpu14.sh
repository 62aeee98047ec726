set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/diag_bench_gap.py > gpurun_out/g14_gap.log 2>&1 || { echo diag failed; tail -20 gpurun_out/g14_gap.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g14_gap.log | grep -v "^\[W"
mkdir -p gpurun_out/prof14
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof14/bench -- python bench.py --steps 50 > gpurun_out/prof14/bench.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof14 -name "*kernel_stats.csv" | head
