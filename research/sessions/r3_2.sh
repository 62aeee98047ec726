# Find the IPC config that hangs at 2 ranks sharing the GPU (progress per config), then the
# pt4 vs pt4w (32x32 MFMA) GEMM A/B on the flagship and long-K shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_2
mkdir -p $O
timeout -k 10 200 python -u scripts/bench_gemm.py --check --tiles pt4,pt4w --shapes 0,2,5,6 --rounds 5 > $O/gemm_pt4w.log 2>&1; rc=$?
grep -v amdgpu.ids $O/gemm_pt4w.log; [ $rc -eq 0 ] || exit $rc
python - > $O/cfgs.json <<'PY'
import json, sys
sys.path.insert(0, "tests")
import test_native_gpu as t
print(json.dumps(t._ipc_cfgs()))
PY
PORT=29655
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_TEST_CFGS="$(cat $O/cfgs.json)" \
  timeout -k 10 170 python -u tests/_ipc_worker.py > $O/ipc2_rank$r.log 2>&1 &
done
wait
tail -5 $O/ipc2_rank0.log; tail -3 $O/ipc2_rank1.log
