# round 6 / 30: the body instantiated per wave group (g1split: no per-phase branch around the vmcnt waits)
# against the product kernel (with stage_ab)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_30
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,g1split --rounds 13 --shapes 65536x1024x1024,8192x8192x8192,65536x1024x4096,65536x1024x512 > $O/ab_g1split_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ab_g1split_bf16.txt; exit 1; }
grep -v "check: max" $O/ab_g1split_bf16.txt
grep "FAIL" $O/ab_g1split_bf16.txt && exit 1
timeout -k 10 300 python -u $L --variants base,g1split --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_g1split_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ab_g1split_mx.txt; exit 1; }
grep -v "check: max" $O/ab_g1split_mx.txt
grep "FAIL" $O/ab_g1split_mx.txt && exit 1
exit 0
