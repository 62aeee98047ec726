# round 5 / 33: the pt4 knob test (each A/B form in a child process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_33
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_native_gpu.py -k "pt4_schedule_knobs" > $O/knob_tests.txt 2>&1 || { echo "failed"; tail -30 $O/knob_tests.txt; exit 1; }
grep -a "PASSED\|FAILED\|passed\|failed" $O/knob_tests.txt | tail -6
