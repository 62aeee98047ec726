# round 5 / 38: operand-traffic ablation under the ONE schedule (is ONE's loss the DMA lead?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_38
mkdir -p $O
DDLB_PT4_ONE=1 timeout -k 10 300 python -u scripts/diag_operand_traffic.py --shapes 65536x1024x1024,65536x1024x8192 > $O/operand_traffic_one.txt 2>&1 || { echo "failed"; tail -20 $O/operand_traffic_one.txt; exit 1; }
cat $O/operand_traffic_one.txt
timeout -k 10 300 python -u scripts/diag_operand_traffic.py --shapes 65536x1024x1024,65536x1024x8192 > $O/operand_traffic_defer.txt 2>&1 || { echo "failed"; tail -20 $O/operand_traffic_defer.txt; exit 1; }
cat $O/operand_traffic_defer.txt
