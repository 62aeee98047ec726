set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/diag_blas.py > gpurun_out/g17_blas.log 2>&1; grep -v amdgpu.ids gpurun_out/g17_blas.log
mkdir -p gpurun_out/prof17
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof17/blas -- python scripts/diag_blas.py > gpurun_out/prof17/blas.log 2>&1; echo "prof rc=$?"
for w in "--warmup 10 --steps 50" "--warmup 200 --steps 50" "--warmup 10 --steps 500" "--warmup 200 --steps 500"; do
  timeout -k 10 200 python bench.py $w > gpurun_out/g17_bench.log 2>&1 || { echo bench failed; tail gpurun_out/g17_bench.log; exit 1; }
  echo "$w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/g17_bench.log)"
done
