# round 5 / 21: write-through store pattern microbenchmark: half 128-B lines per instruction (the
# pt4 bf16 epilogue) vs whole lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_21
mkdir -p $O
timeout -k 10 120 scripts/lab/bin/store_pattern > $O/store_pattern.txt 2>&1 || { echo "failed"; cat $O/store_pattern.txt; exit 1; }
cat $O/store_pattern.txt
