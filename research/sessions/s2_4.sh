set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 0 1 0 1; do
  DDLB_BLAS_TUNE=$t timeout -k 10 120 python scripts/diag_blas_tune.py > gpurun_out/s2_4_tune$t.log 2>&1 || { tail gpurun_out/s2_4_tune$t.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/s2_4_tune$t.log
done
timeout -k 10 300 python bench.py > gpurun_out/s2_4_bench.log 2>&1 || { tail gpurun_out/s2_4_bench.log; exit 1; }
grep -a "^{" gpurun_out/s2_4_bench.log
