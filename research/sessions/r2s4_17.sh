# GEMM lab: pt4 C-store cache policy (nt vs write-through sc1 vs sc1|nt vs sc0|sc1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_17
mkdir -p $O
export LAB_ONLY="pt4,pt4 nt,pt4 wt,pt4 wt nt,pt4 sc01"
timeout -k 10 300 scripts/lab/bin/gemm_lab 65536 1024 1024 > $O/lab_65536.log 2>&1; rc=$?; cat $O/lab_65536.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 scripts/lab/bin/gemm_lab 16384 8192 1024 > $O/lab_16384.log 2>&1; rc=$?; cat $O/lab_16384.log | tail -7; exit $rc
