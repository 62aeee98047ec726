# fp8 / MX-fp8 tiles after the non-temporal store change.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_fp8_tiles.py > gpurun_out/s2_44_fp8.log 2>&1 || { tail gpurun_out/s2_44_fp8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s2_44_fp8.log
