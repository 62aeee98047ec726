set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof24
DDLB_BLAS_TUNE=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof24 -o kt -- python scripts/diag_blas_vs_torch.py > gpurun_out/prof24/log.txt 2>&1; rc=$?; tail -2 gpurun_out/prof24/log.txt; exit $rc
