# round 5 / 8: mid-round validation of the tree (GPU suite, smoke, bench N=1 bf16 / fp8), the
# 2-rank shared-GPU preflight (every RCCL phase reports RCCL's own error, none a timeout), the
# d = 8 budget of the RCCL-fed fused candidates with the stand-in collectives at the CTA cap,
# PMC of the flagship (bf16 pt4 and MX-fp8 vs hipBLASLt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-250 $O/bench_bf16.json
timeout -k 10 400 python bench.py --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-250 $O/bench_fp8.json
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29771 bench.py --gpus 2 --preflight-only --preflight-timeout 60 > $O/preflight2.log 2>&1; rc=$?
grep -a "\[bench\|^{" $O/preflight2.log | cut -c1-700
timeout -k 10 400 python -u scripts/plan_budget.py --world 8 --candidates "coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s8/fused,p2p_pipeline/rccl/fused,coll_pipeline/rccl/s4/fused/cumask,direct/ipc" --rccl-blocks 32 > $O/budget_fused_cap32.txt 2>&1 || { echo "budget failed"; tail -20 $O/budget_fused_cap32.txt; exit 1; }
grep -v "^\[W\|amdgpu.ids" $O/budget_fused_cap32.txt | tail -8
cd /tmp
for spec in "bfloat16 auto" "float8_e4m3fn mx"; do
  set -- $spec
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d /tmp/pmc_$1 -o p -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py -m 65536 -n 1024 -k 1024 --tiles pt4 --hipblaslt --iters 5 --dtype $1 --mode $2 > $GRAFT_REPO_ROOT/$O/pmc_$1.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc_$1.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/pmc_summary.py $(find /tmp/pmc_$1 -name "*.db") --match "" > $GRAFT_REPO_ROOT/$O/pmc_flagship_$1.txt 2>&1
  head -40 $GRAFT_REPO_ROOT/$O/pmc_flagship_$1.txt
done
exit $rc
