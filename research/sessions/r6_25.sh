# round 6 / 25: is the A stream's cost a power-of-two row stride (every concurrent A line at the same low
# address bits)? base / al2 / mrot (K loop rotated by M-block) at K = 4096 vs 4224 and K = 1024 vs 1152
# (rows 8 KB / 8.25 KB and 2 KB / 2.25 KB apart), F.linear beside; MX at K = 4096 vs 4352
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_25
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 400 python -u $L --variants base,al2,mrot --vendor --rounds 9 --shapes 65536x1024x4096,65536x1024x4224,65536x1024x1024,65536x1024x1152 > $O/stride_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/stride_bf16.txt; exit 1; }
cat $O/stride_bf16.txt
timeout -k 10 300 python -u $L --variants base,al2,mrot --dtype mx --rounds 9 --shapes 65536x1024x4096,65536x1024x4352,65536x1024x1024 > $O/stride_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/stride_mx.txt; exit 1; }
cat $O/stride_mx.txt
