# Round 2: do the stream-memop signals dispatch kernels? (kernel trace of scripts/diag_signal_kernels.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r2/sig9
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- python3 scripts/diag_signal_kernels.py > $D/log.txt 2>&1; rc=$?
grep -v amdgpu.ids $D/log.txt | tail -3
find $D -name "*kernel_stats.csv" | head -3 | xargs -r cat | cut -c1-200
exit $rc
