# Round 2: the CLI end to end on the GPU (every slot, both primitives, CSV checked)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests/test_cli_gpu.py -x -v -m gpu --timeout 700 --timeout-method thread > gpurun_out/r2/r2_7_cli.log 2>&1; rc=$?
tail -5 gpurun_out/r2/r2_7_cli.log; exit $rc
