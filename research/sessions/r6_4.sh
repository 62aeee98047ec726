# round 6 / 4: lab -- wave group 0 waits for its fragment reads after the barrier (lgkm_g0), C store policies sc0|nt (3), sc0|sc1|nt (19), sc0|sc1 (17) again with more rounds; rccl_cap at world 1 (the cap of a 2-rank plan) and the diagnostics; 2 ranks sharing the GPU through bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_4
mkdir -p $O
export TMPDIR=/tmp
L=research/lab/pt4_ablate.py
timeout -k 10 200 python -u $L --variants base,lgkm_g0,aux3,aux19,aux17 --rounds 9 --shapes 65536x1024x1024,65536x1024x4096 > $O/ab_cpol_bf16.txt 2>&1 || { echo "ab bf16 failed"; tail -30 $O/ab_cpol_bf16.txt; exit 1; }
cat $O/ab_cpol_bf16.txt
timeout -k 10 120 python -u $L --variants base,lgkm_g0,aux3,aux19,aux17 --dtype mx --rounds 9 --shapes 65536x1024x1024 > $O/ab_cpol_mx.txt 2>&1 || { echo "ab mx failed"; tail -30 $O/ab_cpol_mx.txt; exit 1; }
cat $O/ab_cpol_mx.txt
timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -k "rccl_cap or diagnose" > $O/n1_tests.txt 2>&1 || { echo "tests failed"; grep -v "^  File\|^    " $O/n1_tests.txt | tail -40; exit 1; }
grep -c PASSED $O/n1_tests.txt; tail -2 $O/n1_tests.txt
DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29775 bench.py --gpus 2 --steps 10 --warmup 3 --candidates "direct/ipc,coll_pipeline/ipc/agk32/s4/graph,coll_pipeline/rccl/s4/fused" --preflight-timeout 60 > $O/bench2_shared.log 2>&1 || { echo "bench2 failed"; grep -a "\[bench\|^{\|Error\|error" $O/bench2_shared.log | cut -c1-600 | tail -30; exit 1; }
grep -a "\[bench\|^{" $O/bench2_shared.log | cut -c1-1500 | tail -30
