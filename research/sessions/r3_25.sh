# lab: pt4k with the LDS-DMA instruction offset compensated on the LDS side
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_25
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
LAB_ONLY="pt4 nt,pt4v15,pt4k" timeout -k 10 120 /tmp/gemm_lab 65536 1024 1024 > $O/lab_flagship.log 2>&1 || { tail $O/lab_flagship.log; exit 1; }
cat $O/lab_flagship.log
LAB_ONLY="pt4 nt,pt4v15,pt4k" timeout -k 10 120 /tmp/gemm_lab 8192 8192 8192 > $O/lab_cube.log 2>&1 || { tail $O/lab_cube.log; exit 1; }
cat $O/lab_cube.log
LAB_ONLY="pt4 nt,pt4v15,pt4k" timeout -k 10 120 /tmp/gemm_lab 16384 8192 8192 > $O/lab_row.log 2>&1 || { tail $O/lab_row.log; exit 1; }
cat $O/lab_row.log
