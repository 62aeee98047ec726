# Round 2: graph-mode IPC configurations at world 3 and 4 (one HW queue per process at 4),
# progress per config in gpurun_out/r2/r2_16_w*_rank*.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
CFGS=$(python -c "
import json, sys; sys.path.insert(0, 'tests')
import test_native_gpu as t
print(json.dumps([c for c in t._ipc_cfgs() if c[0].endswith('/graph') and not c[2].get('fused')]))")
for w in 3 4; do
  q=""; [ $w -eq 4 ] && q="GPU_MAX_HW_QUEUES=1"
  for r in $(seq 0 $((w-1))); do
    env $q RANK=$r LOCAL_RANK=$r WORLD_SIZE=$w LOCAL_WORLD_SIZE=$w MASTER_ADDR=127.0.0.1 MASTER_PORT=2960$w \
    DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_TEST_CFGS="$CFGS" \
    timeout -k 10 150 python tests/_ipc_worker.py > gpurun_out/r2/r2_16_w${w}_rank$r.txt 2>&1 &
  done
  wait
  echo "== world $w"; grep -v amdgpu.ids gpurun_out/r2/r2_16_w${w}_rank0.txt | grep "RESULT\|\[rank" | tail -12
done
