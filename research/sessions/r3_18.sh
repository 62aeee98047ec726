# pt4 cycle breakdown (lab copy, nt stores) with s_memtime buckets: flagship and 8192^3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_18
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
LAB_ONLY="pt4 nt,pt4 nt noST,pt4 noDMA,pt4 noLDSrd" LAB_STAMP=1 timeout -k 10 120 /tmp/gemm_lab 65536 1024 1024 > $O/flagship.log 2>&1 || { tail $O/flagship.log; exit 1; }
cat $O/flagship.log
LAB_ONLY="pt4 nt" LAB_STAMP=1 timeout -k 10 120 /tmp/gemm_lab 8192 8192 8192 > $O/cube.log 2>&1 || { tail $O/cube.log; exit 1; }
cat $O/cube.log
