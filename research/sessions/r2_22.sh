# Round 2: which copy_streams configuration crashes? 2 ranks, progress per config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
CFGS=$(python -c "
import json, sys; sys.path.insert(0, 'tests')
import test_native_gpu as t
print(json.dumps([c for c in t._ipc_cfgs() if 'cs2' in c[0]]))")
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_TEST_CFGS="$CFGS" \
  timeout -k 10 150 python tests/_ipc_worker.py > gpurun_out/r2/r2_22_rank$r.txt 2>&1 &
done
wait
grep -v amdgpu.ids gpurun_out/r2/r2_22_rank0.txt | tail -12
