# round 4 / 16: final-tree GEMM table, ours (auto) vs hipBLASLt, every primitive shape, bf16 and fp8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_16
mkdir -p $O
timeout -k 10 500 python -u scripts/bench_gemm.py --tiles auto --rounds 5 --check --json $O/bf16.json > $O/bf16.txt 2>&1 || { echo "bf16 failed"; tail -20 $O/bf16.txt; exit 1; }
grep -v amdgpu.ids $O/bf16.txt
timeout -k 10 500 python -u scripts/bench_gemm.py --dtype float8_e4m3fn --tiles auto --modes mx --rounds 5 --check --json $O/fp8.json > $O/fp8.txt 2>&1 || { echo "fp8 failed"; tail -20 $O/fp8.txt; exit 1; }
grep -v amdgpu.ids $O/fp8.txt
