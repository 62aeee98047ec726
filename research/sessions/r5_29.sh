# round 5 / 29: end-of-round validation of the final tree: whole GPU suite, smoke, bench N=1
# (bf16 flagship, fp8 flagship, config #2), 2-rank shared-GPU preflight
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_29
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
timeout -k 10 400 python bench.py --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-300 $O/bench_fp8.json
timeout -k 10 400 python bench.py -m 8192 -n 1024 -k 8192 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench c2 failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-300 $O/bench_c2_bf16.json
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29771 bench.py --gpus 2 --preflight-only --preflight-timeout 60 > $O/preflight2.log 2>&1; rc=$?
grep -a "\[bench\|^{" $O/preflight2.log | cut -c1-600
exit $rc
