# round 5 / 22: pt4 16-bit C in whole 128-byte lines per store instruction (DPP regroup): GEMM
# correctness, then process-interleaved A/B against the half-line stores (DDLB_PT4_HALF_LINES=1)
# and of nt-only whole-line stores (DDLB_PT4_C_NT=1), bf16 and MX-fp8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_22
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_native_gpu.py -k "gemm or ksplit or split_k or pt4" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 500 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_HALF_LINES --values unset,1 --shapes 0,4,6 --rounds 4 > $O/ab_half_lines_bf16.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab_half_lines_bf16.txt; exit 1; }
grep -A4 "median" $O/ab_half_lines_bf16.txt
timeout -k 10 300 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_HALF_LINES --values unset,1 --shapes 0 --dtype float8_e4m3fn --modes mx --rounds 4 > $O/ab_half_lines_mx.txt 2>&1 || { echo "ab mx failed"; tail -20 $O/ab_half_lines_mx.txt; exit 1; }
grep -A3 "median" $O/ab_half_lines_mx.txt
timeout -k 10 400 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_C_NT --values unset,1 --shapes 0,6 --rounds 4 > $O/ab_c_nt_bf16.txt 2>&1 || { echo "ab nt failed"; tail -20 $O/ab_c_nt_bf16.txt; exit 1; }
grep -A4 "median" $O/ab_c_nt_bf16.txt
