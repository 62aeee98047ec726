# lab: pt4e (halves-1 reads interleaved into MFMA phase A) vs pt4d, raster 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_35
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for shape in "65536 1024 1024" "8192 8192 8192" "16384 8192 8192" "16384 8192 1024"; do
  LAB_RASTER=4 LAB_ONLY="pt4d,pt4e" timeout -k 10 120 /tmp/gemm_lab $shape > $O/l.log 2>&1 || { cat $O/l.log; exit 1; }
  cat $O/l.log
done
