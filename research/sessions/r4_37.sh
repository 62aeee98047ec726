# round 4 / 37: the round's last tree: GPU suite, smoke, bench N=1, 2-rank shared-GPU rehearsal
# of the whole columnwise pool (IPC families; RCCL refuses two ranks per device)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_37
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-250 $O/bench_bf16.json
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29771 bench.py --gpus 2 --steps 10 --warmup 3 --deadline-s 500 > $O/bench2_col.log 2>&1; rc=$?
grep -a "\[bench" $O/bench2_col.log | cut -c1-200; grep -a '^{' $O/bench2_col.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
