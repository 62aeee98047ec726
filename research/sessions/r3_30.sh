# lab: pt4d vs pt4v15 with the product's tile raster (G = 4) at long K, and without
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_30
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for shape in "16384 8192 8192" "8192 8192 8192" "65536 1024 8192" "16384 8192 1024"; do
  LAB_RASTER=4 LAB_ONLY="pt4v15,pt4d" timeout -k 10 120 /tmp/gemm_lab $shape > $O/r4.log 2>&1 || { tail $O/r4.log; exit 1; }
  echo "raster 4:"; grep -v "max|err| = .* ok" $O/r4.log
done
LAB_ONLY="pt4v15,pt4d" timeout -k 10 120 /tmp/gemm_lab 16384 8192 8192 > $O/r0.log 2>&1 || { tail $O/r0.log; exit 1; }
echo "no raster:"; grep -v "max|err| = .* ok" $O/r0.log
