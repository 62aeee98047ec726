set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 python -c "import torch; p=torch.cuda.get_device_properties(0); print(p.name, p.gcnArchName, p.multi_processor_count, p.total_memory//2**30, torch.version.hip)" > gpurun_out/g1_info.log 2>&1 || exit 3
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/g1_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_gemm.py --rounds 3 --iters 10 --json gpurun_out/g1_gemm_bf16.json > gpurun_out/g1_gemm_bf16.log 2>&1 || exit 4
timeout -k 10 200 python scripts/bench_gemm.py --dtype float8_e4m3fn --rounds 3 --iters 10 --tiles auto,256x256 --modes auto,mx --shapes 0,2,6 --json gpurun_out/g1_gemm_fp8.json > gpurun_out/g1_gemm_fp8.log 2>&1 || exit 5
