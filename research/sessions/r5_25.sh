# round 5 / 25: pt4 ONE schedule with a 3-deep A ring (160 KB LDS) behind DDLB_PT4_ONE=1: GEMM tests
# under the knob, then A/B vs DEFER (bf16 and MX)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_25
mkdir -p $O
export TMPDIR=/tmp
DDLB_PT4_ONE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/tests_one.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests_one.txt; exit 1; }
tail -n 1 $O/tests_one.txt
DDLB_PT4_ONE=1 timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 0,2,5,6 --check --rounds 1 --iters 3 --tiles auto > $O/check_one.txt 2>&1 || { echo "check failed"; tail -30 $O/check_one.txt; exit 1; }
grep "check" $O/check_one.txt
timeout -k 10 600 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_ONE --values unset,1 --shapes 0,2,5,6 --rounds 3 > $O/ab_one.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab_one.txt; exit 1; }
grep -A4 "median" $O/ab_one.txt
timeout -k 10 300 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_ONE --values unset,1 --shapes 0,2 --dtype float8_e4m3fn --modes mx --rounds 3 > $O/ab_one_mx.txt 2>&1 || { echo "ab mx failed"; tail -20 $O/ab_one_mx.txt; exit 1; }
grep -A3 "median" $O/ab_one_mx.txt
