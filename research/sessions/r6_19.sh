# round 6 / 19: noprio (MFMA phases without s_setprio 1), second session: flagship, long K, square
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_19
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 500 python -u $L --variants base,noprio --rounds 11 --shapes 65536x1024x1024,65536x1024x4096,65536x1024x8192,16384x8192x8192,8192x8192x8192 > $O/ab_noprio_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_noprio_bf16.txt; exit 1; }
cat $O/ab_noprio_bf16.txt
timeout -k 10 300 python -u $L --variants base,noprio --dtype mx --rounds 11 --shapes 65536x1024x1024,65536x1024x4096,16384x8192x8192 > $O/ab_noprio_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_noprio_mx.txt; exit 1; }
cat $O/ab_noprio_mx.txt
