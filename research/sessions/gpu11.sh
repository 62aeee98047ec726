set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g11_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g11_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
mkdir -p gpurun_out/prof11
timeout -k 10 300 rocprofv3 --selected-regions --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/prof11/win -- python -m ddlb_amd --primitive tp_columnwise -m 65536 -n 1024 -k 1024 --dtype bfloat16 --num-iterations 20 --num-warmups 3 --impl "native;algorithm=default" --impl "pytorch;empty_cache=false" --impl "compute_only;size=unsharded;gemm=torch" --output-csv gpurun_out/prof11/col_{timestamp}.csv > gpurun_out/prof11/win.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof11 -name "*kernel_stats.csv" | head
