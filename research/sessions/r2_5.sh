# Round 2 evidence: kernel-trace stats of the N=1 bench (final measurement, own kernel), one PMC
# pass of the flagship GEMM (own pt4 vs autotuned hipBLASLt), and a 4-rank shared-GPU rehearsal
# of the new IPC candidates.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r2/prof5
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/bench -o kt -- python3 bench.py --algorithm "gemm (world=1)/hip" --steps 50 --warmup 10 > $D/bench.log 2>&1 || { echo bench-prof failed; tail -5 $D/bench.log; exit 1; }
tail -1 $D/bench.log
P="python3 scripts/prof_gemm.py --tiles pt4 --blas --iters 30"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $D/pmc -o p -- $P > $D/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $D/pmc.log; exit 1; }
echo pmc done
export DDLB_ALLOW_SHARED_GPU=1 DDLB_PG_BACKEND=gloo
C="coll_pipeline/ipc/kernel/s4,coll_pipeline/ipc/memcpy/s8,direct/ipc"
GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --steps 10 --warmup 3 --candidate-timeout 60 --candidates "$C" > gpurun_out/r2/r2_5_bench4.log 2>&1; rc=$?
echo "4 ranks rc=$rc"; grep -a "\[bench\]\|^{" gpurun_out/r2/r2_5_bench4.log | cut -c1-250; exit $rc
