# Full GPU suite + smoke + N=1 bench (bf16, fp8, rowwise) + 2/8-rank shared-GPU rehearsals of the
# flagship (validated final runs) with the t8/pt8 GEMMs in every native algorithm.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_19_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2_19_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_19_smoke.log 2>&1 || { tail gpurun_out/s2_19_smoke.log; exit 1; }
tail -1 gpurun_out/s2_19_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s2_19_bench.log 2>&1 || { tail gpurun_out/s2_19_bench.log; exit 1; }
grep -ao '"ms_per_step": [0-9.]*\|"algorithm": "[^"]*"\|"autotune_ms.*' gpurun_out/s2_19_bench.log | tr '\n' ' '; echo
timeout -k 10 300 python bench.py --dtype float8_e4m3fn > gpurun_out/s2_19_fp8.log 2>&1 || { tail gpurun_out/s2_19_fp8.log; exit 1; }
grep -ao '"ms_per_step": [0-9.]*\|"algorithm": "[^"]*"\|"autotune_ms.*' gpurun_out/s2_19_fp8.log | tr '\n' ' '; echo
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
for alg in direct/ipc p2p_pipeline/ipc/push coll_pipeline/ipc/memcpy/s4 default/ipc/kernel; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --algorithm $alg > gpurun_out/s2_19_b2.log 2>&1; rc=$?
  echo "n=2 $alg rc=$rc $(grep -ao '"ms_per_step": [0-9.]*\|"valid": [a-z]*' gpurun_out/s2_19_b2.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 --steps 5 --warmup 2 --algorithm direct/ipc > gpurun_out/s2_19_b8.log 2>&1; rc=$?
echo "n=8 direct rc=$rc $(grep -ao '"ms_per_step": [0-9.]*\|"valid": [a-z]*' gpurun_out/s2_19_b8.log | tr '\n' ' ')"; exit $rc
