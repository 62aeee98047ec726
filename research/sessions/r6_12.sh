# round 6 / 12: where the steady pt4 K-tile's ~2,600 cycles go (2,048 of MFMA issue): the iterations without operand DMA / fragment reads / MFMAs / both DMA and reads (timing only), bf16 long K (stores negligible), flagship and 8192^3; MX flagship
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_12
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 300 python -u $L --variants base,nodma,noread,nomfma,mfmaonly,nostore --rounds 7 --shapes 65536x1024x4096,65536x1024x1024,8192x8192x8192 > $O/ab_loop_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_loop_bf16.txt; exit 1; }
cat $O/ab_loop_bf16.txt
timeout -k 10 200 python -u $L --variants base,nodma,noread,nomfma,mfmaonly,nostore --dtype mx --rounds 7 --shapes 65536x1024x4096,65536x1024x1024 > $O/ab_loop_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_loop_mx.txt; exit 1; }
cat $O/ab_loop_mx.txt
