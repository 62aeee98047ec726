# round 4 / 31: rocprofv3 kernel-trace statistics of the final tree: flagship bf16 (pt4 vs
# hipBLASLt), config #2 shape through the K-split (ops.gemm auto: KS pt4 + reduce), MX flagship
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_31
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/flag -o run -- python3 scripts/prof_gemm.py --tiles pt4 --hipblaslt --iters 30 > $O/flag.log 2>&1 || { echo "prof1 failed"; tail -20 $O/flag.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2 -o run -- python3 scripts/prof_gemm.py -m 8192 -k 8192 --tiles auto --hipblaslt --iters 30 > $O/c2.log 2>&1 || { echo "prof2 failed"; tail -20 $O/c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mx -o run -- python3 scripts/prof_gemm.py --dtype float8_e4m3fn --mode mx --tiles pt4 --iters 30 > $O/mx.log 2>&1 || { echo "prof3 failed"; tail -20 $O/mx.log; exit 1; }
find $O -name "*kernel_stats.csv" | sort
