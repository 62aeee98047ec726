# round 4 / 21: config #2 full GEMM (8192x1024x8192) at the op level: pt4 on 128 CUs, t4, 128x128,
# hipBLASLt (no K split; the plan-level split measured 0.121 ms in r4_20)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_21
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 3,1 --tiles auto,pt4,t4,128x128 --rounds 5 > $O/bf16.txt 2>&1 || { echo "failed"; tail -20 $O/bf16.txt; exit 1; }
grep -v amdgpu.ids $O/bf16.txt
