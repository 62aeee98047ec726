# round 5 / 37: what operand traffic costs the flagship pt4 (timing-only: A / B row pitch 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_37
mkdir -p $O
timeout -k 10 300 python -u scripts/diag_operand_traffic.py --shapes 65536x1024x1024,65536x1024x8192,16384x8192x1024 > $O/operand_traffic_bf16.txt 2>&1 || { echo "failed"; tail -20 $O/operand_traffic_bf16.txt; exit 1; }
cat $O/operand_traffic_bf16.txt
timeout -k 10 300 python -u scripts/diag_operand_traffic.py --dtype float8_e4m3fn --shapes 65536x1024x1024 > $O/operand_traffic_mx.txt 2>&1 || { echo "failed"; tail -20 $O/operand_traffic_mx.txt; exit 1; }
cat $O/operand_traffic_mx.txt
