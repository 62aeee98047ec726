# IPC configs at 3 ranks sharing the GPU (progress per config); PMC of pt4 vs pt4w (32x32 MFMA)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_3
mkdir -p $O
python - > $O/cfgs.json <<'PY'
import json, sys
sys.path.insert(0, "tests")
import test_native_gpu as t
print(json.dumps(t._ipc_cfgs()))
PY
PORT=29657
for r in 0 1 2; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=3 LOCAL_WORLD_SIZE=3 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_TEST_CFGS="$(cat $O/cfgs.json)" \
  timeout -k 10 170 python -u tests/_ipc_worker.py > $O/ipc3_rank$r.log 2>&1 &
done
wait
tail -4 $O/ipc3_rank0.log | cut -c1-3000; tail -2 $O/ipc3_rank1.log; tail -2 $O/ipc3_rank2.log
cd /tmp
for t in pt4 pt4w; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/$O/pmc_$t -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py --tiles $t --iters 10 > $GRAFT_REPO_ROOT/$O/pmc_$t.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/$O/pmcg_$t -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py --tiles $t --iters 10 > $GRAFT_REPO_ROOT/$O/pmcg_$t.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for t in pt4 pt4w; do python scripts/pmc_summary.py $(find $O/pmc_$t $O/pmcg_$t -name "*.db") --match pt4; done
