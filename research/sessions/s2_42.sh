# Kernel-trace durations: product pt4 vs autotuned hipBLASLt vs the lab pt4 (nt) on the flagship.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/kt42
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/prod -o kt -- python3 scripts/prof_gemm.py --tiles pt4 --blas --iters 50 > $D/prod.log 2>&1 || { echo prod failed; tail -5 $D/prod.log; exit 1; }
LAB_ONLY="pt4 nt" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/lab -o kt -- scripts/lab/bin/gemm_lab 65536 1024 1024 > $D/lab.log 2>&1 || { echo lab failed; tail -5 $D/lab.log; exit 1; }
echo done
