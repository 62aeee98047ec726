# round 5 / 30: N>1 flow sanity on the final tree -- 2 ranks sharing the GPU (gloo control plane,
# IPC data plane; RCCL refuses two ranks per GPU): preflight, tuning over the default pool
# (budget 120 s), final timed run with validation
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_30
mkdir -p $O
export TMPDIR=/tmp
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29773 bench.py --gpus 2 --steps 10 --warmup 3 --tune-budget-s 120 --preflight-timeout 60 > $O/bench2_shared.log 2>&1 || { echo "bench2 failed"; grep -a "\[bench\|^{\|Error\|error" $O/bench2_shared.log | tail -30; exit 1; }
grep -a "\[bench\|^{" $O/bench2_shared.log | cut -c1-400 | tail -40
