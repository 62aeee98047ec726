# Round 2 GEMM lab: do chip-wide synchronized C-store bursts cost pt4 time? Odd blocks delayed
# at start (stagger) vs plain pt4 nt vs no stores, flagship shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 300 scripts/lab/bin/gemm_lab 65536 1024 1024 > gpurun_out/r2/r2_4_lab.log 2>&1; rc=$?
cat gpurun_out/r2/r2_4_lab.log | grep -v "max|err|"; exit $rc
