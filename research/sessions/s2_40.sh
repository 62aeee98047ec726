# GEMM lab: q4 (one wave per SIMD, 128x128 wave tiles, accumulators in AGPRs) vs t4 / pt4, with timing ablations.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for shp in "65536 1024 1024" "8192 8192 8192"; do
  tag=$(echo $shp | tr ' ' x)
  timeout -k 10 120 scripts/lab/bin/gemm_lab $shp > gpurun_out/s2_40_$tag.log 2>&1; rc=$?
  cat gpurun_out/s2_40_$tag.log | grep -v "stamps\|block 0\|ideal"; [ $rc -eq 0 ] || exit $rc
done
