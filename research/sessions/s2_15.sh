set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for shp in "65536 1024 1024" "16384 1024 1024" "16384 8192 1024" "65536 1024 8192" "8192 8192 8192"; do
  timeout -k 10 120 scripts/lab/bin/gemm_lab $shp > gpurun_out/s2_15_lab.log 2>&1; rc=$?
  grep -v "^stamps\|^block\|^ideal\|^$" gpurun_out/s2_15_lab.log; [ $rc -eq 0 ] || exit $rc
done
