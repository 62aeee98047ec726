# round 4 / 5: side-stream stall diagnosis (same emulated plan, several binds, priority / caller
# stream / hardware-queue-count variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_side_stream_stall.py > $O/stall_q4.txt 2>&1 || { echo "diag failed"; tail -20 $O/stall_q4.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/stall_q4.txt
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u scripts/diag_side_stream_stall.py > $O/stall_q8.txt 2>&1 || { echo "diag q8 failed"; tail -20 $O/stall_q8.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/stall_q8.txt
timeout -k 10 300 python -u scripts/diag_side_stream_stall.py --candidate coll_pipeline/rccl/s4 --variants base,prio0 > $O/stall_s4.txt 2>&1 || { echo "diag s4 failed"; tail -20 $O/stall_s4.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/stall_s4.txt
