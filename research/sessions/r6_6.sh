# round 6 / 6: DEFER + 3-deep A ring (A staged three K-tiles ahead, 160 KB LDS): GEMM GPU tests (multi-tile cases at nk = 2 / 4 / 6 added), then the lab A/B against the committed kernel (ref) on the flagship, long K and square shapes, bf16 and MX
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_6
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py tests/test_gemm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "pt4 or ksplit or split_k or gemm" > $O/gemm_tests.txt 2>&1 || { echo "tests failed"; grep -v "^  File\|^    " $O/gemm_tests.txt | tail -40; exit 1; }
tail -3 $O/gemm_tests.txt
timeout -k 10 300 python -u $L --variants ref,base --rounds 9 --shapes 65536x1024x1024,65536x1024x4096,65536x1024x8192,8192x8192x8192,16384x8192x8192,65536x1024x512 > $O/ab_ring_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_ring_bf16.txt; exit 1; }
cat $O/ab_ring_bf16.txt
timeout -k 10 200 python -u $L --variants ref,base --dtype mx --rounds 9 --shapes 65536x1024x1024,65536x1024x4096,16384x8192x8192 > $O/ab_ring_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_ring_mx.txt; exit 1; }
cat $O/ab_ring_mx.txt
