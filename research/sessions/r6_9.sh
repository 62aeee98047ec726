# round 6 / 9: PARK -- a quarter of every tile's C stores (4 of 16 per wave) parked in LDS at the tile end and stored after the DMA of the next tile's first K-tile; GEMM GPU tests, then lab A/B: ref (committed), base (park), relax (committed + the exact, looser waits of the first K-tile)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_9
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_gemm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "pt4 or ksplit or split_k or gemm" > $O/gemm_tests.txt 2>&1 || { echo "tests failed"; grep -v "^  File\|^    " $O/gemm_tests.txt | tail -40; exit 1; }
tail -3 $O/gemm_tests.txt
timeout -k 10 300 python -u $L --variants ref,base,relax --rounds 9 --shapes 65536x1024x1024,65536x1024x512,65536x1024x4096,8192x8192x8192 > $O/ab_park_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_park_bf16.txt; exit 1; }
cat $O/ab_park_bf16.txt
timeout -k 10 200 python -u $L --variants ref,base,relax --dtype mx --rounds 9 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_park_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_park_mx.txt; exit 1; }
cat $O/ab_park_mx.txt
