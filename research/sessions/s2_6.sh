set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_s2_6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s2_6 -o bench -- python bench.py --steps 50 --warmup 10 > gpurun_out/prof_s2_6/bench.log 2>&1; rc=$?
echo "rc=$rc"; grep -a "^{" gpurun_out/prof_s2_6/bench.log; find gpurun_out/prof_s2_6 -name "*stats*" | head
