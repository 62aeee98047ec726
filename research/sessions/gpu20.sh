set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "box default GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python scripts/diag_hw_queues.py 8 2>&1 | grep GPU_MAX || exit 1
done
GPU_MAX_HW_QUEUES=4 timeout -k 10 120 python scripts/diag_hw_queues.py 2 2>&1 | grep GPU_MAX || exit 1
