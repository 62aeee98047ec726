set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof5
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5/kt -- python scripts/prof_gemm.py --hipblaslt > gpurun_out/prof5/kt.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/prof5/pmc1 -- python scripts/prof_gemm.py --iters 5 --hipblaslt > gpurun_out/prof5/pmc1.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/prof5/pmc2 -- python scripts/prof_gemm.py --iters 5 --hipblaslt > gpurun_out/prof5/pmc2.log 2>&1 || exit 5
find gpurun_out/prof5 -name "*.csv" | head -20
