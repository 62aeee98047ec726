# round 6 / 2: store-behind pt4 (the tile's C packed into held registers and stored over three
# intervals instead of one) against the committed kernel (lab: ref = HEAD), correctness first;
# stamps of the new kernel; GEMM tests; bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_2
mkdir -p $O
L=research/lab/pt4_ablate.py
timeout -k 10 240 python -u $L --variants ref,base --vendor --rounds 7 --shapes 65536x1024x1024,65536x1024x512,65536x1024x4096,16384x8192x1024 > $O/ab_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_bf16.txt; exit 1; }
cat $O/ab_bf16.txt
timeout -k 10 150 python -u $L --variants ref,base --dtype mx --rounds 7 --shapes 65536x1024x1024,65536x1024x2048 > $O/ab_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_mx.txt; exit 1; }
cat $O/ab_mx.txt
timeout -k 10 120 python -u $L --variants base,stamps --stamp-report --rounds 3 --shapes 65536x1024x1024 > $O/stamps_bf16.txt 2>&1 || { echo "stamps failed"; tail -30 $O/stamps_bf16.txt; exit 1; }
cat $O/stamps_bf16.txt
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_gemm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "pt4 or ksplit or split_k or gemm or cu_holder or rccl_cap or rccl_data_plane or diagnose" > $O/gemm_tests.txt 2>&1 || { echo "tests failed"; tail -60 $O/gemm_tests.txt; exit 1; }
tail -3 $O/gemm_tests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 50 --warmup 10 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cat $O/bench_bf16.json
