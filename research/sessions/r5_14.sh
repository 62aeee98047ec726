# round 5 / 14: f32 pt4 / t4 stores regrouped with v_permlane32_swap (64 contiguous bytes per row
# per instruction): GEMM + K-split tests, K-split forms A/B, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_reduce_gpu.py tests/test_native_gpu.py -k "gemm or ksplit or split_k or reduce" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --tiles pt4 --shapes 8192x1024x8192,4096x1024x8192,8192x1024x4096 > $O/ksplit_forms_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ksplit_forms_bf16.txt; exit 1; }
grep -v "^  check.* ok$" $O/ksplit_forms_bf16.txt
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --tiles pt4 --dtype float8_e4m3fn --shapes 8192x1024x8192,4096x1024x8192 > $O/ksplit_forms_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ksplit_forms_mx.txt; exit 1; }
grep -v "^  check.* ok$" $O/ksplit_forms_mx.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ks -- python3 -u scripts/ab_ksplit_forms.py --shapes 8192x1024x8192 --only 'ks2' --rounds 2 > $O/ks_prof.txt 2>&1 || { echo "prof failed"; tail -30 $O/ks_prof.txt; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-6 "$f" | cut -c1-160 | head -12
