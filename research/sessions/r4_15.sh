# round 4 / 15: per-tile fixed cost vs per-K-tile work of pt4 (bf16, MX-fp8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_15
mkdir -p $O
timeout -k 10 400 python -u scripts/diag_tile_overhead.py > $O/fit.txt 2>&1 || { echo "fit failed"; tail -20 $O/fit.txt; exit 1; }
grep -v amdgpu.ids $O/fit.txt
