# lab only: pt4k (K-half split) vs pt4v15 vs pt4, read-swap stamps
# GEMM numerics suite, GEMM vs hipBLASLt (bf16 + MX), bench N=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_24
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/lab/gemm_lab.hip -o /tmp/gemm_lab > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
LAB_ONLY="pt4 nt,pt4v15,pt4v15 AfirstBsecond,pt4k" LAB_STAMP=k timeout -k 10 120 /tmp/gemm_lab 65536 1024 1024 > $O/lab_flagship.log 2>&1 || { tail $O/lab_flagship.log; exit 1; }
cat $O/lab_flagship.log
LAB_ONLY="pt4 nt,pt4v15,pt4k" LAB_STAMP=x timeout -k 10 120 /tmp/gemm_lab 8192 8192 8192 > $O/lab_cube.log 2>&1 || { tail $O/lab_cube.log; exit 1; }
cat $O/lab_cube.log
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1; rc=$?; tail -3 $O/gemm_tests.log; grep -a "FAILED\|Timeout" $O/gemm_tests.log | head; [ $rc -eq 0 ] || exit $rc
