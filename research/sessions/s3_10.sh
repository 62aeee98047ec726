# Session 3: scripts/scaling_curve.py end to end at world 1 (fp8, BASELINE config #5 dtype).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/scaling_curve.py --gpus 1 --steps 50 --warmup 10 --timeout 500 --out gpurun_out/s3_10_scaling_fp8.md -- --dtype float8_e4m3fn > gpurun_out/s3_10_scaling.log 2>&1; rc=$?
echo "scaling rc=$rc"; cat gpurun_out/s3_10_scaling_fp8.md; exit $rc
