# round 6 / 11: HOLD + PARK -- 8 of a wave's 16 C stores leave beside the next tile's MFMAs (4 held in registers, stored after the DMA of K-tile 0's load phases; 4 parked in LDS, stored after K-tile 1's MFMA phases); GEMM GPU tests, lab A/B ref (committed: park in K-tile 0) vs base
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_11
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_gemm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "pt4 or ksplit or split_k or gemm" > $O/gemm_tests.txt 2>&1 || { echo "tests failed"; grep -v "^  File\|^    " $O/gemm_tests.txt | tail -40; exit 1; }
tail -3 $O/gemm_tests.txt
timeout -k 10 300 python -u $L --variants ref,base --rounds 11 --shapes 65536x1024x1024,65536x1024x512,65536x1024x2048,16384x1024x1024,8192x8192x8192 > $O/ab_hold_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_hold_bf16.txt; exit 1; }
cat $O/ab_hold_bf16.txt
timeout -k 10 200 python -u $L --variants ref,base --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x2048,65536x1024x512 > $O/ab_hold_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_hold_mx.txt; exit 1; }
cat $O/ab_hold_mx.txt
