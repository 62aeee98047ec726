# round 5 / 12: f32-partial K-split (reduce rounds once): reduce kernel tests, forms A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_reduce_gpu.py > $O/reduce_tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/reduce_tests.txt; exit 1; }
tail -3 $O/reduce_tests.txt
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --tiles pt4,256x128 --shapes 8192x1024x8192,4096x1024x8192,8192x1024x4096 > $O/ksplit_forms_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ksplit_forms_bf16.txt; exit 1; }
grep -v "^  check.* ok$" $O/ksplit_forms_bf16.txt
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --tiles pt4,256x128 --dtype float8_e4m3fn --shapes 8192x1024x8192,4096x1024x8192,8192x1024x4096 > $O/ksplit_forms_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ksplit_forms_mx.txt; exit 1; }
grep -v "^  check.* ok$" $O/ksplit_forms_mx.txt
