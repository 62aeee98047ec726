# round 5 / 6: diagnose the in-launch K-split reduction's wrong outputs (S = 2, batched path);
# gated-GEMM placement diagnostic; flagship C-store cache-policy A/B (DDLB_PT4_CAUX)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_6
mkdir -p $O
export TMPDIR=/tmp
export DDLB_CHILD_INIT_METHOD=tcp://127.0.0.1:29533
timeout -k 10 120 python -u scripts/diag_ksr.py > $O/diag_ksr.txt 2>&1 || { echo "diag_ksr failed"; tail -20 $O/diag_ksr.txt; }
grep "{" $O/diag_ksr.txt | cut -c1-400
timeout -k 10 120 python -u scripts/diag_ksr.py --S 4 > $O/diag_ksr4.txt 2>&1 || { echo "diag_ksr4 failed"; tail -20 $O/diag_ksr4.txt; }
grep "{" $O/diag_ksr4.txt | cut -c1-400
unset DDLB_CHILD_INIT_METHOD
timeout -k 10 400 python -u scripts/diag_gate_placement.py --configs 32:32,32:64,32:256,24:8,24:32,24:256,16:16,16:64 > $O/gate_placement.txt 2>&1 || { echo "diag failed"; tail -20 $O/gate_placement.txt; exit 1; }
cat $O/gate_placement.txt
timeout -k 10 500 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_CAUX --values 18,16,19,2 --shapes 0,6 --rounds 3 > $O/ab_caux_bf16.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab_caux_bf16.txt; exit 1; }
tail -12 $O/ab_caux_bf16.txt
