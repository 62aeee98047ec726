# round 5 / 15: in-launch K-split with an agent release before each done count; public op's
# split = f32 partials + one-rounding reduce; 20 checked calls per form
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py tests/test_gemm_gpu.py -k "ksplit or split_k" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 400 python -u scripts/ab_ksplit_forms.py --tiles pt4 --checks 20 --shapes 8192x1024x8192,4096x1024x8192,8192x1024x4096 > $O/ksplit_forms_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ksplit_forms_bf16.txt; exit 1; }
cat $O/ksplit_forms_bf16.txt
timeout -k 10 400 python -u scripts/ab_ksplit_forms.py --tiles pt4 --checks 20 --dtype float8_e4m3fn --shapes 8192x1024x8192,4096x1024x8192 > $O/ksplit_forms_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ksplit_forms_mx.txt; exit 1; }
cat $O/ksplit_forms_mx.txt
