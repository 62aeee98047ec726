# Round 2: the other BASELINE configs through bench.py at N=1 (validated tuning): fp8 flagship
# (config #5 dtype) and tp_rowwise m=16384 n=8192 k=8192 (config #3 shape).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 400 python bench.py --dtype float8_e4m3fn > gpurun_out/r2/r2_11_fp8.log 2>&1; rc=$?
grep -a "\[bench\]\|^{" gpurun_out/r2/r2_11_fp8.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > gpurun_out/r2/r2_11_row.log 2>&1; rc=$?
grep -a "\[bench\]\|^{" gpurun_out/r2/r2_11_row.log | cut -c1-400; exit $rc
