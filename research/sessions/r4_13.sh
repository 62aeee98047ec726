# round 4 / 13: pt4 start-stagger A/B (half the CUs half a tile out of phase)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/ab_pt4_stagger.py --ns 0,2000,4000,7000,12000 --rounds 7 > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py -k "rccl_fed_gated or direct_store" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29733 bench.py --gpus 2 --preflight-only > $O/preflight2.json 2> $O/preflight2.err; rc=$?
cat $O/preflight2.json | cut -c1-900; [ $rc -le 1 ] || exit $rc
