# round 6 / 7: lab -- desynchronized tile phases: workgroup slots started late (stagG_Dk) so fewer CUs end their tiles (and burst their C stores) at the same time; bf16 and MX flagship, K = 4096
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_7
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
V=base,stag2_3k,stag2_6k,stag2_12k,stag4_3k,nostore
timeout -k 10 240 python -u $L --variants $V --rounds 9 --shapes 65536x1024x1024,65536x1024x4096,8192x8192x8192 > $O/ab_stag_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_stag_bf16.txt; exit 1; }
cat $O/ab_stag_bf16.txt
timeout -k 10 200 python -u $L --variants $V --dtype mx --rounds 9 --shapes 65536x1024x1024 > $O/ab_stag_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_stag_mx.txt; exit 1; }
cat $O/ab_stag_mx.txt
