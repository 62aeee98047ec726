# round 6 / 8: is the pt4 C-store interval a per-CU or a chip-wide limit? per-barrier stamps with 32 / 128 / 256 workgroups of one tile each against the flagship's 256 x 4 tiles (bf16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_8
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 200 python -u $L --variants base,stamps,nostore --stamp-report --rounds 3 --shapes 2048x1024x1024,8192x1024x1024,16384x1024x1024,65536x1024x1024 > $O/stamps_grid.txt 2>&1 || { echo "stamps failed"; tail -30 $O/stamps_grid.txt; exit 1; }
cat $O/stamps_grid.txt
