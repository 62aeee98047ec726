set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_native_gpu.py tests/test_models.py -m gpu -x -q > gpurun_out/g12_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g12_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/bench_overhead.py > gpurun_out/g12_overhead.log 2>&1; echo "overhead rc=$?"; grep -v amdgpu.ids gpurun_out/g12_overhead.log | grep -v "^\[" 
