# round 5 / 1: N>1 safety changes: CTA-capped communicator (world-1 RCCL-fed gated GEMM incl. the
# p2p s=1 table form), tile_order 3 refusal on plain A, the HW-queue-pool premise of gemm_first,
# masked-stream flags / priority, preflight with every phase executed (2 ranks sharing the GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py -k "queue_pools or own_shard_needs or rccl_fed_gated or rccl_data_plane or preflight_shared or cumask" > $O/tests.txt 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $O/tests.txt | tail -30; exit 1; }
grep -E "passed|failed|one HW queue|cu-masked" $O/tests.txt | tail -8
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
