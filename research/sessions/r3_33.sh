# lab: pt4v15 schedule knobs (static priority, no priority, LDS-DMA before the fragment reads), raster 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_33
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
V="pt4v15,pt4v15 staticprio,pt4v15 noprio,pt4v15 dmafirst,pt4d"
for shape in "65536 1024 1024" "8192 8192 8192"; do
  LAB_RASTER=4 LAB_ONLY="$V" timeout -k 10 120 /tmp/gemm_lab $shape > $O/l.log 2>&1 || { tail $O/l.log; exit 1; }
  grep -v "max|err| = .* ok" $O/l.log
done
