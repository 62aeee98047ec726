# Round 2 lab: LDS-DMA / store bytes per clock per CU vs pieces in flight (scripts/lab/dma_rate.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 120 scripts/lab/bin/dma_rate > gpurun_out/r2/r2_6_dma_rate.log 2>&1; rc=$?
cat gpurun_out/r2/r2_6_dma_rate.log; exit $rc
