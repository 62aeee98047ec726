set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/s2_26_bench$i.log 2>&1 || { tail gpurun_out/s2_26_bench$i.log; exit 1; }
  grep -a "\[bench\]" gpurun_out/s2_26_bench$i.log; grep -ao '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gemm": "[^"]*"' gpurun_out/s2_26_bench$i.log | tr '\n' ' '; echo
done
