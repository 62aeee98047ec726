# PMC counters of the lab kernels on the flagship shape (one counter pass per run, each run alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc18
for v in "ring2 dmaAC" t8 pt8; do
  tag=$(echo $v | cut -d' ' -f1)
  LAB_ONLY="$v" timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE -d gpurun_out/pmc18/$tag -o p -- scripts/lab/bin/gemm_lab 65536 1024 1024 > gpurun_out/pmc18/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 gpurun_out/pmc18/$tag.log; exit 1; }
  echo "$tag done"
done
