# PMC counters of the product GEMMs on the flagship: our pt4 vs hipBLASLt (autotuned algorithm).
# One counter pass per run; kernel-trace stats in their own run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmc28
mkdir -p $D
P="python3 scripts/prof_gemm.py --tiles pt4 --blas --iters 30"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt -o kt -- $P > $D/kt.log 2>&1 || { echo kt failed; tail -5 $D/kt.log; exit 1; }
i=0
for pass in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_SMEM SQ_WAVES GRBM_COUNT" \
            "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $D/p$i -o p -- $P > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
  echo "pass $i done"
done
