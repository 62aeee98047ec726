# Session 3: smoke + N=1 bench on the final tree (GPU suite ran on this .so in s3_9).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_11_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/s3_11_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s3_11_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/s3_11_bench.log; exit $rc
