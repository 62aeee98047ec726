# round 6 / 1: the pt4 epilogue priced on today's kernel (lab variants: no C stores, C stores
# into L2 only), a per-barrier cycle profile (stamps), then the GEMM tests after the round-6
# retirements (ONE / in-launch K-split / half lines / nt knob) and bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_1
mkdir -p $O
L=research/lab/pt4_ablate.py
timeout -k 10 200 python -u $L --variants base,nostore,l2store --vendor --shapes 65536x1024x1024,65536x1024x512,65536x1024x4096 > $O/ablate_bf16.txt 2>&1 || { echo "ablate bf16 failed"; tail -30 $O/ablate_bf16.txt; exit 1; }
cat $O/ablate_bf16.txt
timeout -k 10 120 python -u $L --variants base,nostore,l2store --dtype mx --shapes 65536x1024x1024,65536x1024x2048 > $O/ablate_mx.txt 2>&1 || { echo "ablate mx failed"; tail -30 $O/ablate_mx.txt; exit 1; }
cat $O/ablate_mx.txt
timeout -k 10 120 python -u $L --variants base,stamps --stamp-report --rounds 3 --shapes 65536x1024x1024 > $O/stamps_bf16.txt 2>&1 || { echo "stamps failed"; tail -30 $O/stamps_bf16.txt; exit 1; }
cat $O/stamps_bf16.txt
timeout -k 10 120 python -u $L --variants base,stamps --stamp-report --rounds 3 --dtype mx --shapes 65536x1024x1024 > $O/stamps_mx.txt 2>&1 || { echo "stamps mx failed"; tail -30 $O/stamps_mx.txt; exit 1; }
cat $O/stamps_mx.txt
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_gemm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "pt4 or ksplit or split_k or gemm or cu_holder or rccl_cap or rccl_data_plane" > $O/gemm_tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/gemm_tests.txt; exit 1; }
tail -3 $O/gemm_tests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 50 --warmup 10 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cat $O/bench_bf16.json
