set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g7_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g7_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g7_smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 300 python bench.py > gpurun_out/g7_bench1.log 2>&1; echo "bench1 rc=$?"; tail -1 gpurun_out/g7_bench1.log
DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --candidate-timeout 90 > gpurun_out/g7_bench2.log 2>&1; echo "bench2 rc=$?"; grep '^{' gpurun_out/g7_bench2.log
