# round 4 / 7: pt4 DEFER C-store slack (knob 0 = new counts, 1 = round-3 counts) A/B + race
# screens; MX with nt (not write-through) C stores as a second variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/ab_gemm_knob.py --knobs 0,1 > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
DDLB_PT4_NT_STORES=1 timeout -k 10 400 python -u scripts/ab_gemm_knob.py --knobs 0,1 --rounds 5 > $O/ab_nt.txt 2>&1 || { echo "ab nt failed"; tail -20 $O/ab_nt.txt; exit 1; }
echo "== nt stores"; cat $O/ab_nt.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "pt4 or t8_kernel or grouped or long_k" > $O/gemm.txt 2>&1 || { echo "gemm tests failed"; tail -30 $O/gemm.txt; exit 1; }
tail -n 2 $O/gemm.txt
