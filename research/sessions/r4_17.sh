# round 4 / 17: does HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) cut the
# reference-default timing's per-iteration launch + completion round trip?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_17
mkdir -p $O
timeout -k 10 300 python -u scripts/diag_harness_overhead.py --schedule auto,spin > $O/default.txt 2>&1 || { echo "diag failed"; tail -20 $O/default.txt; exit 1; }
echo "kernarg default:"; cat $O/default.txt
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u scripts/diag_harness_overhead.py --schedule auto,spin > $O/devkernarg.txt 2>&1 || { echo "diag2 failed"; tail -20 $O/devkernarg.txt; exit 1; }
echo "HIP_FORCE_DEV_KERNARG=1:"; cat $O/devkernarg.txt
