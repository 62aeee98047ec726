# pt4v (VALU-free load phases) lab variants vs pt4: correctness, timing, stamps (flagship, 8192^3, 16384x8192x8192)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_22
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
V="pt4 nt,pt4v0,pt4v1,pt4v3,pt4v7,pt4v15"
LAB_ONLY="$V" LAB_STAMP=v timeout -k 10 120 /tmp/gemm_lab 65536 1024 1024 > $O/flagship.log 2>&1 || { tail $O/flagship.log; exit 1; }
cat $O/flagship.log
LAB_ONLY="$V" LAB_STAMP=v timeout -k 10 120 /tmp/gemm_lab 8192 8192 8192 > $O/cube.log 2>&1 || { tail $O/cube.log; exit 1; }
cat $O/cube.log
LAB_ONLY="pt4 nt,pt4v15" timeout -k 10 120 /tmp/gemm_lab 16384 8192 8192 > $O/row.log 2>&1 || { tail $O/row.log; exit 1; }
cat $O/row.log
