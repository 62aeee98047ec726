# round 5 / 11: few-tile long-K GEMM forms (unsplit pt4 / 256x128 / 128x256 vs K-split pt4 with
# the reduce kernel or the in-launch reduce), bf16 and MX-fp8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --shapes 8192x1024x8192,4096x1024x8192,4096x2048x8192,8192x1024x4096 > $O/ksplit_forms_bf16.txt 2>&1 || { echo "bf16 failed"; tail -30 $O/ksplit_forms_bf16.txt; exit 1; }
cat $O/ksplit_forms_bf16.txt
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --dtype float8_e4m3fn --shapes 8192x1024x8192,4096x1024x8192,4096x2048x8192,8192x1024x4096 > $O/ksplit_forms_mx.txt 2>&1 || { echo "mx failed"; tail -30 $O/ksplit_forms_mx.txt; exit 1; }
cat $O/ksplit_forms_mx.txt
