# lab: pt4v15 ablations (timing only) on the flagship and MX-less 8192^3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_28
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
V="pt4v15,pt4v15 noST,pt4v15 noLDSrd,pt4v15 noMFMA,pt4v15 noDMA,pt4v15 noDMA noST,pt4v15 MFMA only"
LAB_ONLY="$V" timeout -k 10 120 /tmp/gemm_lab 65536 1024 1024 > $O/lab_flagship.log 2>&1 || { tail $O/lab_flagship.log; exit 1; }
cat $O/lab_flagship.log
LAB_ONLY="$V" timeout -k 10 120 /tmp/gemm_lab 8192 8192 8192 > $O/lab_cube.log 2>&1 || { tail $O/lab_cube.log; exit 1; }
cat $O/lab_cube.log
