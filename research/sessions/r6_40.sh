# round 6 / 40: 2 ranks sharing the GPU through bench.py on the final tree (stage_ab + SPLIT): preflight,
# autotune of the first N>1 candidates, final run, diagnostics
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_40
mkdir -p $O
export TMPDIR=/tmp
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29775 bench.py --gpus 2 --steps 10 --warmup 3 --candidates "direct/ipc,coll_pipeline/ipc/agk32/s4/graph,coll_pipeline/rccl/s4/fused" --preflight-timeout 60 > $O/bench2_shared.log 2>&1 || { echo "bench2 failed"; grep -a "\[bench\|^{\|Error\|error" $O/bench2_shared.log | cut -c1-600 | tail -30; exit 1; }
grep -a "\[bench" $O/bench2_shared.log | cut -c1-300
grep -a "^{" $O/bench2_shared.log | cut -c1-700
