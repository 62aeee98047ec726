# round 4 / 24: tile choice for 128-tile short-K GEMMs (8192x1024x1024, the d = 8 shard / s = 8
# stage GEMM): every candidate kernel vs hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_24
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 1 --tiles auto,pt4,t4,t8,256x128,128x256,128x128,i128,256x128w4 --rounds 7 --check > $O/bf16.txt 2>&1 || { echo "bf16 failed"; tail -20 $O/bf16.txt; exit 1; }
grep -v amdgpu.ids $O/bf16.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --dtype float8_e4m3fn --shapes 1 --tiles auto,pt4,t4,256x128,128x128 --modes mx,auto --rounds 7 > $O/fp8.txt 2>&1 || { echo "fp8 failed"; tail -20 $O/fp8.txt; exit 1; }
grep -v amdgpu.ids $O/fp8.txt
