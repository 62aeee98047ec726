set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for q in 4 8 16; do
  for ns in 1 3 7; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python scripts/diag_queue_blocking.py $ns 2>&1 | grep GPU_MAX || exit 1
  done
done
